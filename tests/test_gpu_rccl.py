"""RCCL and libhbam in one process on one GPU (the driver's N>1 bench runs
every rank this way): torch.cuda.set_device + init_process_group("nccl"),
then libhbam's own HIP pipeline on the same device, with all_gather_object
and a CUDA-tensor all_reduce between two decodes of the same split.  Run in a
child process so the process group never outlives the test."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import json, os, socket, sys
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import torch
import torch.distributed as dist
with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
import hbam
import orc
from hbam import synth
data, info = synth.make_bam(300000, as_numpy=True)
path = os.path.join(TMP, "rccl.bam")
data.tofile(path)
out = {}
with hbam.BamFile(path=path, device=0, window_bytes=8 << 20) as f:
    first = f.header()["first_record_voff"]
    a = f.decode_span_device(first, (1 << 64) - 1, digest=True)
    g = [None]
    dist.all_gather_object(g, (a["records"], a["key_digest"], a["voff_digest"]))
    t = torch.tensor([float(a["records"]), 2.5], dtype=torch.float64, device="cuda:0")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    dist.barrier()
    b = f.decode_span_device(first, (1 << 64) - 1, digest=True)
    ent = f.splitting_entries(first, (1 << 64) - 1, 4096, 0)
r, _ = orc.scan(data, threads=4)
out.update(records=[a["records"], b["records"], r["records"], info["n_records"]],
           key_digest=[a["key_digest"], b["key_digest"], r["key_digest"]],
           voff_digest=[a["voff_digest"], b["voff_digest"], r["voff_digest"]],
           gathered=list(g[0]), reduced=t.tolist(), windows=a["windows"], entries=[ent[0], len(ent[1])])
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
"""


def test_rccl_process_group_beside_libhbam(tmp_path):
    code = f"ROOT = {ROOT!r}\nTMP = {str(tmp_path)!r}\n" + CHILD
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, NCCL_DEBUG="WARN"))
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1]
    r = json.loads(line[len("RESULT "):])
    n = r["records"][0]
    assert r["records"] == [n, n, n, n]
    assert len(set(r["key_digest"])) == 1 and len(set(r["voff_digest"])) == 1
    assert r["gathered"] == [n, r["key_digest"][0], r["voff_digest"][0]]
    assert r["reduced"] == [float(n), 2.5]
    assert r["windows"] > 1  # 8 MiB windows: the multi-window path
    assert r["entries"] == [n, n // 4096]
