"""The C-ABI library loads on a CPU-only host, exports every symbol
include/avdb.h declares, and its host-side entry points (context, formatting)
agree with the oracle.  No kernel is launched here."""

import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from annotatedvdb_amd import _native as N
from annotatedvdb_amd.chromosomes import CHROM_NAMES, length_table
from oracle import avdb_oracle as O

HEADER = os.path.join(ROOT, "include", "avdb.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(avdb_[a-z0-9_]+)\s*\(", txt, re.M)))


def test_header_matches_binding_list():
    assert declared_symbols() == sorted(N.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.avdb_abi_version() == N.ABI_VERSION == 2


def test_nm_dynamic_exports():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (avdb_[a-z0-9_]+)$", out, re.M))
    assert set(declared_symbols()) <= exported


@pytest.fixture(scope="module")
def host_ctx():
    lib = N.load_library()
    lens = length_table()
    arr = (ctypes.c_uint32 * len(lens))(*lens)
    h = ctypes.c_void_p()
    assert lib.avdb_ctx_create(-1, arr, len(lens), ctypes.byref(h)) == 0  # host-only context
    yield lib, h
    lib.avdb_ctx_destroy(h)


def test_ctx_argument_checks(host_ctx):
    lib, h = host_ctx
    assert lib.avdb_ctx_n_chrom(h) == 25
    nb = ctypes.c_uint32()
    assert lib.avdb_l8_bin_count(h, ctypes.byref(nb)) == 0
    assert nb.value == O.l8_offsets(length_table())[-1] == 6189
    bad = ctypes.c_void_p()
    assert lib.avdb_ctx_create(-1, None, 0, ctypes.byref(bad)) == N.AVDB_EINVAL
    assert b"chromosome" in lib.avdb_last_error()
    zero = (ctypes.c_uint32 * 2)(5, 0)
    assert lib.avdb_ctx_create(-1, zero, 2, ctypes.byref(bad)) == N.AVDB_EINVAL
    # null context / arrays are rejected before any GPU work
    assert lib.avdb_bin_assign(None, None, None, None, 1, None, None, None, None, None) == N.AVDB_EINVAL
    assert lib.avdb_bin_assign(h, None, None, None, 1, None, None, None, None, None) == N.AVDB_EINVAL
    assert lib.avdb_bin_assign(h, None, None, None, 0, None, None, None, None, None) == 0  # n == 0 no-op
    ws = ctypes.c_size_t()
    assert lib.avdb_pk_dedup_workspace_size(1000, ctypes.byref(ws)) == 0 and ws.value >= 8 * 1000


def test_format_paths_match_oracle(host_ctx):
    lib, h = host_ctx
    rng = np.random.default_rng(5)
    lens = length_table()
    n = 20000
    chrom = rng.integers(0, 25, n).astype(np.uint8)
    L = np.asarray(lens, dtype=np.int64)[chrom]
    s = (rng.random(n) * L).astype(np.int64) + 1
    e = np.minimum(L, s + (10 ** rng.uniform(0, 7, n)).astype(np.int64))
    codes, status = O.bin_codes_np(chrom, s, e, lens)
    out = np.empty(n * 90, dtype=np.uint8)
    offs = np.empty(n + 1, dtype=np.uint64)
    assert lib.avdb_format_bin_paths(h, chrom.ctypes.data, codes.ctypes.data, n, out.ctypes.data,
                                     out.size, offs.ctypes.data) == 0
    raw = out.tobytes()
    for i in range(0, n, 7):
        got = raw[int(offs[i]):int(offs[i + 1])].decode()
        assert got == O.format_bin_path(CHROM_NAMES[chrom[i]], int(codes[i]))
    buf = ctypes.create_string_buffer(128)
    k = lib.avdb_format_bin_path(h, int(chrom[0]), int(codes[0]), buf, 128)
    assert buf.raw[:k].decode() == O.format_bin_path(CHROM_NAMES[chrom[0]], int(codes[0]))
    assert lib.avdb_format_bin_path(h, 0, 0xFFFFFFFF, buf, 128) == N.AVDB_EINVAL
    assert lib.avdb_format_bin_path(h, 0, int(codes[0]), buf, 3) == N.AVDB_ERANGE
    # output-capacity check of the batch form
    assert lib.avdb_format_bin_paths(h, chrom.ctypes.data, codes.ctypes.data, n, out.ctypes.data,
                                     10, offs.ctypes.data) == N.AVDB_ERANGE


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from annotatedvdb_amd.engine import Engine
    with pytest.raises(N.NativeUnavailable):
        Engine()
    from annotatedvdb_amd.bin_index import BinIndex
    with pytest.raises(N.NativeUnavailable):
        BinIndex(None, verbose=False)


def test_hist_allgather_argument_checks(host_ctx):
    """The RCCL entry points refuse bad arguments before touching RCCL or a GPU;
    the workspace is (world + 1) per-rank slots of padded histogram + counters."""
    lib, ctx = host_ctx
    sz = ctypes.c_size_t()
    assert lib.avdb_hist_allgather_workspace_size(8, 6189, 32, ctypes.byref(sz)) == 0
    assert sz.value == 9 * ((4 * 6189 + 7) // 8 * 8 + 8 * 32)
    assert lib.avdb_hist_allgather_workspace_size(0, 1, 1, ctypes.byref(sz)) == N.AVDB_EINVAL
    assert lib.avdb_hist_allgather(ctx, None, None, 0, None, 0, None, None, None, 0, None) == N.AVDB_EINVAL
    comm = ctypes.c_void_p()
    assert lib.avdb_rccl_comm_init(ctx, 2, 2, b"x" * 128, ctypes.byref(comm)) == N.AVDB_EINVAL
    assert lib.avdb_rccl_comm_destroy(None) == 0
