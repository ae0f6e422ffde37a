"""Profile the per-call drop-in path (parse_variant / find_bin_index) on the
host alone: the K8h entry needs no GPU, so an engine stand-in with a device -1
context and a numpy arena runs the product's per-call code here.  Development
tool (build container); the box numbers come from ``bench.py --workload dropin``.

    python tools/percall_profile.py [--prof]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from annotatedvdb_amd import _native as N  # noqa: E402
from annotatedvdb_amd import engine as E  # noqa: E402
from annotatedvdb_amd.chromosomes import length_table  # noqa: E402


class HostArena(E.SmallPrep):
    def _alloc(self, total):
        self._np = np.zeros(total + 64, dtype=np.uint8)
        return (self._np.ctypes.data + 63) & ~63

    def close(self):
        self._ptr = None


class HostEngine:
    """Just what SmallPrep / BinIndex / the loader's per-call path touch."""

    def __init__(self):
        self.lib = N.load_library()
        self.lengths = length_table()
        arr = (ctypes.c_uint32 * 25)(*self.lengths)
        h = ctypes.c_void_p()
        N.check("ctx", self.lib.avdb_ctx_create(-1, arr, 25, ctypes.byref(h)))
        self.ctx = h
        self.device = None
        self._small = None

    def line_host(self):
        if getattr(self, "_lh", None) is None:
            self._lh = E.LineHost(self)
        return self._lh

    def small(self):
        if self._small is None:
            self._small = HostArena(self)
            self._small.mode = "host"
        return self._small


def main():
    from annotatedvdb_amd import synth, bin_index, loaders
    eng = HostEngine()
    def bi_init(self, *a, **k):
        self._engine, self._lengths, self._currentBin, self._verbose, self._k1h = eng, eng.lengths, {}, False, None
    bin_index.BinIndex.__init__ = bi_init
    ld = loaders.VCFVariantLoader("dbSNP")
    ld.initialize_pk_generator("GRCh38", None)
    ld.initialize_bin_indexer(None)
    ld.set_algorithm_invocation_id(1)
    ld.initialize_copy_sql()
    lines = synth.vcf_text(3000, seed=17).decode().splitlines()
    for x in lines[:50]:
        ld.parse_variant(x)
    if "--prof" in sys.argv:
        import cProfile
        import pstats
        pr = cProfile.Profile(); pr.enable(); [ld.parse_variant(x) for x in lines]; pr.disable(); pr.dump_stats("/tmp/pv.prof")
        pstats.Stats("/tmp/pv.prof").sort_stats("cumulative").print_stats(30)
        return
    def best(fn, items, reps=5):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            for x in items:
                fn(x)
            ts.append((time.perf_counter() - t0) / len(items) * 1e6)
        return min(ts)
    t = best(ld.parse_variant, lines)
    from oracle import avdb_oracle as O
    from annotatedvdb_amd.chromosomes import GRCH38_LENGTHS
    pbi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    lens = length_table()
    tp = best(lambda x: O.load_line(x, lens, bin_index=pbi), lines)
    print(f"port load_line {tp:.1f} us/line")
    bi = bin_index.BinIndex(None)
    rng = np.random.default_rng(9)
    L = eng.lengths[21]
    st = rng.integers(1, L - 1_100_000, 3000)
    sp = (10 ** rng.uniform(np.log10(16_000), 6, 3000)).astype(np.int64)
    t1 = time.perf_counter()
    for s, e in zip(st.tolist(), (st + sp).tolist()):
        bi.find_bin_index("22", s, e)
    tm = (time.perf_counter() - t1) / 3000 * 1e6
    pbi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    t2 = time.perf_counter()
    for s_, e_ in zip(st.tolist(), (st + sp).tolist()):
        pbi.find_bin_index("22", s_, e_)
    tpm = (time.perf_counter() - t2) / 3000 * 1e6
    print(f"parse_variant {t:.1f} us/line   find_bin_index miss {tm:.2f} us (port {tpm:.2f})")


if __name__ == "__main__":
    main()
