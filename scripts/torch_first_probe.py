"""Does libhbam see the GPU after torch has used it (developer probe)?  torch
and libhbam share one libamdhip64.so.7 (same soname: whichever loads first
serves both).  Prints hbam.device_count() after each torch step."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import ctypes as C  # noqa: E402

import torch  # noqa: E402

import hbam  # noqa: E402


def report(tag):
    n = C.c_int(-1)
    hip = C.CDLL("libamdhip64.so.7")
    rc = hip.hipGetDeviceCount(C.byref(n))
    last = hip.hipGetLastError()
    print(f"{tag}: hbam.device_count={hbam.device_count()} hipGetDeviceCount rc={rc} n={n.value} last={last}",
          flush=True)


report("import")
torch.cuda.set_device(0)
x = torch.ones(4, device="cuda")
torch.cuda.synchronize()
report("small tensor")
h = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
d = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
d.copy_(h, non_blocking=True)
h.copy_(d, non_blocking=True)
torch.cuda.synchronize()
report("1 GiB pinned copies")
del h, d
torch.cuda.empty_cache()
report("after empty_cache")
data = bytes(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "test.bam"),
                  "rb").read())
with hbam.BamFile(data, device=0) as f:
    print("decoded", len(f.decode_all()["key"]), flush=True)
