#!/usr/bin/env python3
"""Attribution probes for k_keyed_onepass (round 6): patched copies of
avdb_keys.hip built OUTSIDE the tree's sources (/tmp), linked with the in-tree
objects into _lib/var/libavdb_<name>.so.  Each probe drops one part of the pass
(its output is wrong; timing only): nolb (no look-back wait: offsets from 0),
nostore (no K2 output stores), norender (no key/path tiles), tpw2 / tpw1
(2 / 1 tiles per wave), w1 / w2 (1 / 2 waves per workgroup), w1t2 / w2t2."""
import os, re, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "annotatedvdb_amd/csrc/avdb_keys.hip")).read()
P = {
    "nolb": [("    group_lookback(P.lb, P.hdr, g, ak, ap, &xk, &xp);", "    xk = xp = 0;")],
    "nostore": [("      __builtin_nontemporal_store(e, P.end + i);\n      __builtin_nontemporal_store(cd, P.code + i);\n"
                 "      if (P.status) P.status[i] = uint8_t(st);\n      if (P.long_codes) P.long_codes[i] = uint8_t(long_code(cur[k].r, cur[k].a, P.max_seq_len));\n"
                 "      if (P.keep) P.keep[i] = 1;\n", "      (void)e;\n")],
    "norender": [("  key_tile(A, cur[0], w0, run_k, run_p, kimg, pimg, hp, lane);\n", "  if (run_k == 12345) key_tile(A, cur[0], w0, run_k, run_p, kimg, pimg, hp, lane);\n"),
                 ("  if constexpr (TPW > 1) key_tile(", "  if constexpr (TPW > 1) if (run_k == 12345) key_tile("),
                 ("  if constexpr (TPW > 2) key_tile(", "  if constexpr (TPW > 2) if (run_k == 12345) key_tile("),
                 ("  if constexpr (TPW > 3) key_tile(", "  if constexpr (TPW > 3) if (run_k == 12345) key_tile(")],
    "tpw2": [], "tpw1": [], "w1": [], "w2": [], "w1t2": [], "w2t2": [],
    "t1np": [], "t2np": [], "t2p": [], "t4np": [],
}
flags = {"tpw2": ["-DAVDB_OP_TPW=2"], "tpw1": ["-DAVDB_OP_TPW=1"], "w1": ["-DAVDB_OP_WAVES=1"],
         "w2": ["-DAVDB_OP_WAVES=2"], "w1t2": ["-DAVDB_OP_WAVES=1", "-DAVDB_OP_TPW=2"],
         "w2t2": ["-DAVDB_OP_WAVES=2", "-DAVDB_OP_TPW=2"],
         "t1np": ["-DAVDB_OP_TPW=1", "-DAVDB_OP_PIPE=0"], "t2np": ["-DAVDB_OP_TPW=2", "-DAVDB_OP_PIPE=0"],
         "t2p": ["-DAVDB_OP_TPW=2", "-DAVDB_OP_PIPE=1"], "t4np": ["-DAVDB_OP_TPW=4", "-DAVDB_OP_PIPE=0"]}
for name in (sys.argv[1:] or P):
    s = src
    for a, b in P[name]:
        assert a in s, (name, a[:50])
        s = s.replace(a, b)
    d = f"/tmp/probe/{name}"
    os.makedirs(d, exist_ok=True)
    f = os.path.join(d, "avdb_keys.hip")
    open(f, "w").write(s)
    obj = f"/tmp/probe/{name}.o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-w",
                           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "annotatedvdb_amd/csrc"),
                           *flags.get(name, []), "-c", f, "-o", obj])
    objs = [os.path.join(ROOT, "annotatedvdb_amd/_lib/obj", o) for o in sorted(os.listdir(os.path.join(ROOT, "annotatedvdb_amd/_lib/obj")))
            if o.endswith(".o") and o != "avdb_keys.o"]
    os.makedirs(os.path.join(ROOT, "annotatedvdb_amd/_lib/var"), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                           os.path.join(ROOT, f"annotatedvdb_amd/_lib/var/libavdb_{name}.so"), *objs, obj])
    print("built", name)
