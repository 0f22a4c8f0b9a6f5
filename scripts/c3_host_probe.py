"""C3-shaped file (header segment + repeated 10M-record segment) decoded from
the mapped file window by window, per library variant (HBAM_LIB)."""
import os, sys, time, subprocess
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "hadoop-bam_amd"))
if len(sys.argv) > 2 and sys.argv[1] == "--child":
    import hbam
    path = sys.argv[2]
    with hbam.BamFile(path=path) as f:
        first = f.header()["first_record_voff"]
        for i in range(2):
            t = time.perf_counter()
            st = f.decode_span_device(first, (1 << 64) - 1, timing=False, digest=True)
            dt = time.perf_counter() - t
            print(f"{os.path.basename(os.environ.get('HBAM_LIB', 'libhbam.so'))} pass {i}: {dt:.3f} s "
                  f"{st['records']} records, windows {st['windows']}, key_xor {st['key_xor']:#x}", flush=True)
    sys.exit(0)
import numpy as np
from hbam import synth
gb = float(sys.argv[1])
r = 10_000_000
head, _ = synth.make_bam_segment(2 * r, 0, r, with_header=True, eof_block=False, seed=11)
body, _ = synth.make_bam_segment(2 * r, r, 2 * r, with_header=False, eof_block=False, seed=11)
k = max(1, int(gb * 1e9) // body.nbytes)
EOF_BLK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
path = f"/dev/shm/c3probe_{os.getpid()}.bam"
try:
    with open(path, "wb") as fh:
        fh.write(head.tobytes())
        b = body.tobytes()
        for _ in range(k):
            fh.write(b)
        fh.write(EOF_BLK)
    del head, body, b
    print(f"file {os.path.getsize(path) / 1e9:.1f} GB", flush=True)
    for lib in sys.argv[2:]:
        env = dict(os.environ, HBAM_LIB=os.path.abspath(lib))
        rc = subprocess.run([sys.executable, "-u", __file__, "--child", path], env=env, timeout=240).returncode
        if rc != 0:
            print(f"{lib}: rc {rc}", flush=True)
            break
finally:
    os.unlink(path)
