import os
import sys

import pytest

# torch first: it bundles its own libamdhip64.so.7 (ROCm 7.0), the same soname
# as the system ROCm runtime libpech_crc32c.so links, so whichever loads first
# serves the whole process.  With the library's runtime first, torch's device
# query fails; with torch's first, both work (as in bench.py and smoke()).
import torch  # noqa: F401,E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")
