"""CPU oracle (TEST INFRASTRUCTURE ONLY — the checker, never the product).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package.  ``avdb_oracle`` is the Python/numpy restatement,
``c_oracle()`` loads the plain-C restatement (``avdb_oracle.c``) built by
``make -C oracle``.
"""

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
C_LIB = os.path.join(_HERE, "_build", "libavdb_oracle.so")
CPUBASE_LIB = os.path.join(_HERE, "_build", "libavdb_cpubase.so")
_c = None
_cb = None


def build_c_oracle() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return C_LIB


def c_oracle():
    """ctypes handle of the C oracle (built on first use if gcc is present)."""
    global _c
    if _c is None:
        if not os.path.exists(C_LIB):
            build_c_oracle()
        lib = ctypes.CDLL(C_LIB)
        P, SZ, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        lib.avdb_oracle_bin_assign.argtypes = [P, P, P, SZ, P, I, P, P]
        lib.avdb_oracle_record_prep.argtypes = [P, P, P, P, P, P, SZ, P, I, P, P, P, P]
        lib.avdb_oracle_dedup_grouped.argtypes = [P, P, P, P, P, P, P, SZ, P]
        lib.avdb_oracle_dedup_grouped.restype = ctypes.c_uint64
        lib.avdb_oracle_sha512.argtypes = [P, SZ, P]
        lib.avdb_oracle_vrs_digest.argtypes = [P, P, P, P, P, P, SZ, ctypes.c_uint32, ctypes.c_char_p, I, P, P]
        lib.avdb_oracle_primary_keys.argtypes = [P, P, P, P, P, P, P, P, SZ, ctypes.c_uint32, P, P]
        lib.avdb_oracle_primary_keys.restype = SZ
        lib.avdb_oracle_bin_paths.argtypes = [P, P, SZ, P, P]
        lib.avdb_oracle_bin_paths.restype = SZ
        _c = lib
    return _c


def cpubase():
    """ctypes handle of the OpenMP comparator (``cpu_baseline.c``: the C oracle's
    per-record functions at -O3 over all host cores) — bench.py's second
    ``cpu_baseline`` leg only."""
    global _cb
    if _cb is None:
        if not os.path.exists(CPUBASE_LIB):
            build_c_oracle()
        lib = ctypes.CDLL(CPUBASE_LIB)
        P, SZ, I, U32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32
        lib.avdb_cpubase_bin_assign.argtypes = [P, P, P, SZ, P, I, P, P, I]
        lib.avdb_cpubase_keyed.argtypes = [P, P, P, P, P, P, P, SZ, P, I, U32, ctypes.c_char_p, P, P, P, P, P, SZ,
                                           SZ, I]
        lib.avdb_cpubase_keyed.restype = ctypes.c_uint64
        _cb = lib
    return _cb
