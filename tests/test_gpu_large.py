"""C3-shaped parity at scale: an ~8.5 GB BAM (header segment + body segments
of 3 distinct record runs, each repeated an odd number of times in shuffled
order -- bench.py's C3 builder at a smaller size) read through the drop-in
call (hbam_open by path, hbam_decode_span in 1M-record batches over 1 GiB
windows) and compared with orc_scan_records on the host's cores: every key
and every voff in order, an order-sensitive digest of each of the 11 fixed
fields, the crc32 of every record's rest bytes back to back, and the
.splitting-bai at g = 4096 byte for byte (SplittingBAMIndexer.java:248-290)."""
import os
import time
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _OneRank:
    world, rank = 1, 0

    @staticmethod
    def all_gather(obj):
        return [obj]

    @staticmethod
    def barrier():
        pass


def test_8gb_file_keys_and_voffs_match_oracle(tmp_path):
    import bench
    import hbam
    import orc
    path = os.path.join(bench.scratch_dir(), f"hbam_large_{os.getpid()}.bam")
    try:
        t = time.time()
        meta = bench.build_c3_file(path, _OneRank, 8.5, seg_records=2_000_000)
        n = meta["records"]
        print(f"built {meta['compressed_bytes']} B, {n} records in {time.time() - t:.1f}s", flush=True)
        assert meta["compressed_bytes"] >= 8_000_000_000
        keys = np.empty(n, np.int64)
        voffs = np.empty(n, np.uint64)
        fields = {f: [] for f in orc._ScanResult.FIELDS}  # [(records, digest)] per batch
        rest_crc, rest_bytes = 0, 0
        k = 0
        with hbam.BamFile(path=path, window_bytes=1 << 30) as f:
            v, end = f.header()["first_record_voff"], (1 << 64) - 1
            while v < end:
                r = f.decode_span(v, end, max_records=1 << 20)
                m = len(r["key"])
                if m == 0:
                    break
                keys[k:k + m] = r["key"]
                voffs[k:k + m] = r["voff"]
                for fn in fields:
                    fields[fn].append(orc.digest_np(r[fn]))
                # the batch's data holds exactly its records' rests, in order
                assert int(r["rest_off"][0]) == 0 and len(r["data"]) == int(r["rest_len"].sum(dtype=np.uint64))
                rest_crc = zlib.crc32(r["data"], rest_crc)
                rest_bytes += len(r["data"])
                k += m
                v = r["next_voff"]
            read = f.bytes_read()
            sbi = f.splitting_index(4096)
        assert k == n
        # about one pass over the file: 1 GiB windows overlap by a record's blocks
        assert read <= meta["compressed_bytes"] * 1.02 + (2 << 20), (read, meta["compressed_bytes"])
        data = np.memmap(path, np.uint8, mode="r")
        d, ok, ov = orc.scan_records(data, n, threads=bench.host_cores())
        assert d["rc"] == 0 and d["records"] == n
        np.testing.assert_array_equal(voffs, ov)
        np.testing.assert_array_equal(keys, ok)
        for fn, parts in fields.items():
            assert orc.digest_concat(parts) == (n, d["field_digest"][fn]), fn
        assert (rest_bytes, rest_crc) == (d["rest_bytes"], d["rest_crc"])
        di, want_sbi = orc.scan(data, threads=bench.host_cores(), mode="index", granularity=4096)
        assert di["rc"] == 0 and sbi == want_sbi
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
