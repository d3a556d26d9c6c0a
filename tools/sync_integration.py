"""Write integration/pech_crc32c_msgr.patch into INTEGRATION.md's ```diff
block, so the document shows exactly the patch tests/test_dropin_build.py
applies and compiles against the reference."""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
doc_path = os.path.join(REPO, "INTEGRATION.md")
doc = open(doc_path).read()
body = open(os.path.join(REPO, "integration", "pech_crc32c_msgr.patch")).read()
start = doc.index("```diff\n") + len("```diff\n")
end = doc.index("```", start)
open(doc_path, "w").write(doc[:start] + body + doc[end:])
print("INTEGRATION.md: patch block updated (%d lines)" % body.count("\n"))
