"""pech_amd -- MI355X-native (gfx950) CRC32C message-checksum path for pech.

The product is libpech_crc32c.so (C-ABI: include/crc32c.h drop-in for
/root/reference/include/crc32c.h:88, plus include/pech_crc32c.h batch/device
API).  This package is its Python mirror for tests and benchmarks.
"""
from .crc32c import (  # noqa: F401
    AsyncCrc, Pages, async_devices, crc32c_concat, set_cpu_max, set_flat_max, stats,
    Crc32cError, crc32c, crc32c_batch, crc32c_combine, crc32c_shift, crc32c_tensors, dev_batch_async,
    dev_batch_small_async, dev_batch_ws_async, dev_copy_batch_ws_async, dev_copy_batch_small_async, make_descs, workspace_bytes, shard_ranges, timing, timing_read, timing_samples, version, F_HOST, F_DEVICE, F_PINNED, F_ALL_DEVICES,
)
