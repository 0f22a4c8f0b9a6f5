"""Rehearsal of bench.py's multi-GPU sequence on one GPU: torch.cuda.set_device +
init_process_group("nccl") (RCCL), then libhbam's own HIP pipeline in the same
process, then RCCL collectives on the timing tensors -- the mix of torch's HIP
runtime and libhbam's that the driver's N>1 scaling run relies on."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd")]
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
import hbam
from hbam import synth

data, info = synth.make_bam(200000, as_numpy=True)
g = hbam.Gpu(0)
g.load(data)
st = g.run(timing=True)
torch.cuda.synchronize()
dist.barrier()
t = torch.tensor([1.5], dtype=torch.float64, device="cuda:0")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
tot = torch.tensor([float(info["uncompressed"]), float(st["records"])], dtype=torch.float64, device="cuda:0")
dist.all_reduce(tot)
print("ok", st["records"], t.item(), tot.tolist(), flush=True)
g.close()
dist.destroy_process_group()
