"""CPU: libhbam.so loads, exports every entry point include/hbam.h declares,
its scalar key helpers match the oracle, and the product fails loudly without
a GPU (no CPU fallback)."""
import ctypes as C

import numpy as np
import pytest

import hbam
import orc
import py_oracle


def test_exports_every_declared_symbol():
    names = hbam.exported_symbols_from_header()
    assert len(names) >= 25
    lib = C.CDLL(hbam.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version():
    assert hbam.lib().hbam_abi_version() == 6


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors have the layout a C compiler gives include/hbam.h."""
    import os
    import subprocess
    src = tmp_path / "layout.c"
    src.write_text("""#include <stdio.h>
#include <stddef.h>
#include "hbam.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(hbam_opts), offsetof(hbam_opts, window_bytes),
         sizeof(hbam_batch), offsetof(hbam_batch, next_voff), offsetof(hbam_batch, status),
         sizeof(hbam_gpu_stats), sizeof(hbam_header_info));
  return 0;
}
""")
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(hbam.HEADER_PATH))
    subprocess.check_call(["gcc", "-I", inc, "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [C.sizeof(hbam.Opts), hbam.Opts.window_bytes.offset, C.sizeof(hbam.Batch),
                   hbam.Batch.next_voff.offset, hbam.Batch.status.offset, C.sizeof(hbam.GpuStats),
                   C.sizeof(hbam.HeaderInfo)]


def test_unknown_stringency_is_an_argument_error(test_bam):
    # hadoopbam.samheaderreader.validation-stringency takes STRICT / LENIENT / SILENT only
    with pytest.raises(hbam.HbamError) as e:
        hbam.BamFile(test_bam, stringency=7)
    assert e.value.code == hbam.E_ARG


def test_write_time_index_granularity_checked_first():
    with pytest.raises(hbam.HbamError) as e:
        hbam.splitting_index_for_records([1, 2, 3], 0, 100)
    assert e.value.code == hbam.E_ARG


def test_static_keys_match_reference_semantics():
    # BAMRecordReader.getKey0 / getKey (BAMRecordReader.java:114-121)
    assert hbam.get_key0(1, 99) == 0x0000000100000063
    assert hbam.get_key(1, 100) == 0x0000000100000063
    assert hbam.get_key0(3, -1) == -1
    assert hbam.get_key0(0x7FFFFFFF, -2) == -2
    assert hbam.get_key0(-1, 5) == (-1 << 32) | 5


def test_murmur_helper_matches_oracles():
    rng = np.random.default_rng(1)
    for n in list(range(0, 34)) + [255, 256, 257, 4096]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 123, -1):
            assert hbam.murmurhash3(b, seed) == orc.murmurhash3(b, seed) == py_oracle.murmurhash3(b, seed)


def test_no_gpu_fails_loudly(test_bam):
    if hbam.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(hbam.HbamError) as e:
        hbam.BamFile(test_bam)
    assert e.value.code == hbam.E_DEVICE
    with pytest.raises(hbam.HbamError):
        hbam.Gpu(0)
    # the BGZF write path has no CPU path either
    with pytest.raises(hbam.HbamError) as e:
        hbam.bgzf_compress(b"ACGT" * 1000)
    assert e.value.code == hbam.E_DEVICE


def test_bgzf_compress_argument_errors():
    # checked before any device work: block_lens must cover the payload, block_size 1..65536
    with pytest.raises(hbam.HbamError) as e:
        hbam.bgzf_compress(b"ACGT" * 10, block_lens=[39])
    assert e.value.code == hbam.E_ARG
    with pytest.raises(hbam.HbamError) as e:
        hbam.bgzf_compress(b"ACGT" * 10, block_size=65537)
    assert e.value.code == hbam.E_ARG
    # an explicit empty block list does not cover a non-empty payload
    with pytest.raises(hbam.HbamError) as e:
        hbam.bgzf_compress(b"ACGT" * 10, block_lens=[])
    assert e.value.code == hbam.E_ARG
