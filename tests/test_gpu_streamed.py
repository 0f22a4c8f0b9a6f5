"""End-to-end pass from host memory (hbam_gpu_run_streamed): the compressed
file is copied to HBM in pieces while the blocks of landed pieces are located
and inflated.  Results must be identical to the device-resident pass (which
the parity tests pin against the oracle) and to the oracle itself."""
import numpy as np
import pytest

import hbam
import orc
from hbam import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw,piece", [
    (dict(n_records=60000), 1 << 20),                          # ~18 pieces, blocks cut at every piece end
    (dict(n_records=40000, block_payload=4096), 1 << 20),      # small blocks: many per piece
    (dict(n_records=8000, level=0), 1 << 20),                  # stored blocks (csize ~ 64 KiB)
    (dict(n_records=300, mode="long"), 3 << 20),               # records spanning blocks and pieces
    (dict(n_records=20000), 64 << 20),                         # one piece
])
def test_streamed_matches_resident_and_oracle(kw, piece):
    data, info = synth.make_bam(as_numpy=True, **kw)
    g = hbam.Gpu(0)
    buf = hbam.PinnedBuffer(data.nbytes)
    try:
        g.load(data)
        st0 = g.run()
        k0, v0 = g.fetch(st0["records"])
        buf.array[:] = data
        st = g.run_streamed(buf.ptr, data.nbytes, piece)
        assert st["status"] == 0
        assert st["records"] == st0["records"] == kw["n_records"]
        assert st["n_blocks"] == info["blocks"]
        assert st["inflated_bytes"] == info["uncompressed"]
        k1, v1 = g.fetch(st["records"])
        np.testing.assert_array_equal(k1, k0)
        np.testing.assert_array_equal(v1, v0)
        # and a second streamed pass over the same buffers (state reset)
        st2 = g.run_streamed(buf.ptr, data.nbytes, piece)
        k2, _ = g.fetch(st2["records"])
        np.testing.assert_array_equal(k2, k0)
    finally:
        buf.close()
        g.close()
    s = orc.Stream(data.tobytes())
    rc, want = s.decode_all()
    assert rc == 0
    np.testing.assert_array_equal(k1, want["key"])
    np.testing.assert_array_equal(v1, want["voff"])
