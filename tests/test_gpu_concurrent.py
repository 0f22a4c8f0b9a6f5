"""Many readers in one process (a Spark executor runs a BAMRecordReader per
task thread, README.md:36-39; SURVEY 8b "re-entrant across ctxs"): 8 threads,
each with its own context on the same file and GPU, decode different splits
at once with close / reopen churn, every batch checked against the oracle.
ctypes drops the GIL for the duration of each C call, so the contexts really
run concurrently (their streams, caches and error strings)."""
import threading

import numpy as np
import pytest

import hbam
import orc
from hbam import synth

pytestmark = pytest.mark.gpu

THREADS = 8


def test_eight_contexts_decode_concurrently(tmp_path):
    data, _ = synth.make_bam(200000, block_payload=16384)
    path = str(tmp_path / "c.bam")
    open(path, "wb").write(data)
    s = orc.Stream(data)
    size = len(data)
    n_splits = 16
    step = -(-size // n_splits)
    starts = [i * step for i in range(n_splits)]
    lengths = [min(step, size - a) for a in starts]
    with hbam.BamFile(path=path) as f:
        splits = f.get_splits(starts, lengths)
    want = []
    for vs, ve in splits:
        rc, r = s.decode_span(vs, ve)
        assert rc == 0
        want.append(r)
    errors = []

    def worker(t):
        try:
            for rnd in range(3):
                # small windows: every split spans several; batches of 7000 records
                with hbam.BamFile(path=path, window_bytes=1 << 20) as f:
                    for j in range(t, len(splits), THREADS):
                        vs, ve = splits[j]
                        parts = list(f.iter_batches(vs, ve, 7000))
                        keys = np.concatenate([p["key"] for p in parts]) if parts else np.zeros(0, np.int64)
                        voffs = np.concatenate([p["voff"] for p in parts]) if parts else np.zeros(0, np.uint64)
                        if not (np.array_equal(keys, want[j]["key"]) and np.array_equal(voffs, want[j]["voff"])):
                            errors.append((t, rnd, j, "batches"))
                        st = f.decode_span_device(vs, ve, digest=True)
                        kd = orc.digest(want[j]["key"].astype(np.uint64))
                        if st["records"] != len(want[j]["key"]) or st["key_digest"] != kd:
                            errors.append((t, rnd, j, "device"))
                # a failure with no context to hold its message (hbam_last_error(NULL)):
                # each thread reads its own (thread-local) message
                dev = 1000 + 10 * t + rnd
                try:
                    hbam.Codec(device=dev)
                    errors.append((t, rnd, "opened a missing device"))
                except hbam.HbamError as e:
                    if f"no HIP device {dev}" not in str(e):
                        errors.append((t, rnd, "foreign error message", str(e)))
        except Exception as e:  # reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=200)
    assert not any(x.is_alive() for x in th)
    assert errors == []
