#!/usr/bin/env python3
"""Benchmark: variants binned(+keyed)/s on MI355X, with HBM-roofline accounting.

Default workload (N=1): BASELINE.json configs[1] — 100 M synthetic GRCh38 SNVs,
point-position bin assignment (K1 ``avdb_bin_assign`` with the fused L8
histogram + level/status counters).  A *step* is one pass of the hot path over
the GPU's whole resident batch.  Per-GPU work is fixed (weak scaling): each rank
owns a length-balanced set of 64 Mb genome pieces (``annotatedvdb_amd.shard``)
and its own 100 M records; ranks never exchange records.  The only collective
is one RCCL all-gather of the per-rank L8 histograms + counters at the end of the
job, inside the timed region.

Other workloads (``--workload``): c3 spans (1e8, K1 with end), c5 ADSP-style
alleles (2.5e7 per GPU: K2 record prep + K3 grouped dedup + K4 long-key digests).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c5]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "variants binned+keyed/sec (node) at 1/2/4/8 MI355X; % of HBM roofline"

WORKLOADS = {
    "c1": dict(n=1_100_000, desc="C1: chr22 1.1 M records (88% SNV / 6% ins / 6% del, seed 1; BASELINE "
                                 "configs[0], the config the reference CPU path is quoted on): K2 end + bin, "
                                 "K3 keep-first dedup, K7 primary-key + ltree-path text",
               bytes_per=None, kernel="whole C1 step (K2 + K3 + K7)"),
    "c2": dict(n=100_000_000, desc="C2: synthetic GRCh38 SNVs, point-position bin assignment "
                                   "(BASELINE configs[1]); K1 bin_assign + L8 histogram",
               bytes_per=9, kernel="k_bin_assign4"),
    "c3": dict(n=100_000_000, desc="C3: synthetic indels/SVs, spans <= 1 Mb, smallest enclosing bin "
                                   "(BASELINE configs[2]); K1 bin_assign + L8 histogram",
               bytes_per=13, kernel="k_bin_assign4"),
    "c4": dict(n=125_000_000, desc="C4: dbSNP-scale mix (90% SNV / 8% indel <= 50 bp / 2% <= 1 Mb), "
                                   "1e9 over 8 GPUs = 1.25e8 per GPU (BASELINE configs[3]); K1 + L8 histogram",
               bytes_per=13, kernel="k_bin_assign4"),
    "c4k": dict(n=125_000_000, desc="C4 keyed: dbSNP-scale 1e9 records over 8 GPUs = 1.25e8 per GPU as VCF "
                                     "alleles (90% SNV / 8% indel <= 48 bp / 2% long, rsids; synth.dbsnp_alleles, "
                                     "BASELINE configs[3] + north_star's 'bin paths and primary keys for 1B'): K2 end "
                                     "+ bin, K3 dedup, K4 long-key digests, K7 primary-key + ltree-path text",
                bytes_per=None, kernel="whole C4k step (K2 + K3 + K4 + K7)"),
    "c5": dict(n=25_000_000, desc="C5: ADSP-style alleles, end inference + bin + grouped PK dedup + "
                                  "long-allele key digests (BASELINE configs[4])",
               bytes_per=None, kernel="k_record_prep"),
    "vcf": dict(n=8_388_608, desc="SURVEY 8f rank 1: dbSNP-shaped VCF text -> per-ALT record SoA on the "
                                  "GPU (K0 tokenizer: line split + field parse + multi-allelic explode)",
                bytes_per=None, kernel="avdb_vcf (whole tokenizer)"),
}
WORKLOADS["dropin"] = dict(
    n=0, desc="drop-in per-call latency (INTEGRATION.md 1): BinIndex.find_bin_index on sorted C1 records "
              "(cache hits) and on > 15.6 kb spans (every call a miss), VCFVariantLoader.parse_variant per "
              "line as load_vcf_file.py:112 calls it, and the batched paths per line",
    bytes_per=None, kernel=None)
WORKLOADS["load"] = dict(
    n=8_388_608, desc="SURVEY 8f ranks 1-3: dbSNP-shaped VCF text -> COPY rows + .mapping lines on the GPU "
                      "(K0 tokenize, K2 end+bin, K5 display attributes/FREQ/keys/paths as text)",
    bytes_per=None, kernel="k_vcf_format<write>")
VCF_TILE = 1 << 19  # distinct synthetic lines, tiled on the device to n
CEILING_LOG = os.path.join(ROOT, "profiles", "hbm_ceiling_r05.jsonl")  # tools/hbm_ceiling.hip on MI355X


def stream_ceiling(test: str, pmc_path: str, kernel_ms: float):
    """A kernel's measured HBM bytes per launch (request-size counters, `pmc_path`) over its time,
    against the best stream rate tools/hbm_ceiling.hip measured for the same read/write mix (any
    access form of the committed runs): how close the kernel is to what HBM delivers for its byte
    mix, not to the spec."""
    if not (os.path.exists(CEILING_LOG) and os.path.exists(pmc_path)):
        return None
    rates = [json.loads(l)["TBps"] for l in open(CEILING_LOG)
             if l.startswith("{") and json.loads(l)["test"].startswith(test)]
    pk = json.load(open(pmc_path))
    if not rates or "hbm_bytes_per_launch" not in pk:
        return None
    ceil = 1e3 * max(rates)  # the best access form measured (unroll, nontemporal, occupancy)
    ach = pk["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9
    return {"mix": test, "measured_traffic_GBps": ach, "ceiling_GBps": ceil, "frac": ach / ceil,
            "read_bytes": pk.get("hbm_read_bytes"), "write_bytes": pk.get("hbm_write_bytes"),
            "source": os.path.relpath(pmc_path, ROOT) + " bytes / stage time; ceiling: profiles/hbm_ceiling_r05.jsonl "
                      "(tools/hbm_ceiling.hip, 16-B grid-stride streams, read:write 1:3, best access form)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--n", type=int, default=None, help="records per GPU (default: config size)")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="target seconds per CPU worker")
    ap.add_argument("--keyed", default="auto", choices=["auto", "on", "off"],
                    help="also run the keyed C4k step and attach it as 'keyed' (auto: with the default c2 line)")
    ap.add_argument("--dry-run", action="store_true", help="rank plumbing only (gloo, CPU): the launcher test")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step as a captured HIP graph (auto: the launch-bound C1 step)")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# CPU baseline: the reference-structured port (oracle) on the host cores
# ---------------------------------------------------------------------------
_SAMPLE = None
_TABLE = None


def _cpu_load_worker(k):
    """Reference-structured load path (oracle.load_line: VcfEntryParser-style parse,
    per-alt key / end / cached bin lookup / FREQ / display attributes / COPY row +
    .mapping line) over this worker's lines."""
    from oracle import avdb_oracle as O
    from annotatedvdb_amd.chromosomes import length_table
    lines = _SAMPLE[k]
    bi = O.PortBinIndex(_TABLE)
    lens = length_table()
    t0 = time.perf_counter()
    recs = 0
    for ln in lines:
        _, _, rows = O.load_line(ln, lens, bin_index=bi)
        recs += len(rows)
    return recs, time.perf_counter() - t0


def _cpu_vcf_worker(k):
    """Reference-structured VCF tokenize (oracle.parse_vcf_line: VcfEntryParser
    parse_entry + get_variant, vcf_parser.py:76-169) and the per-ALT explode with
    the '.' skip (vcf_variant_loader.py:273-280) over this worker's lines."""
    from oracle import avdb_oracle as O
    lines = _SAMPLE[k]
    t0 = time.perf_counter()
    recs = 0
    for ln in lines:
        v = O.parse_vcf_line(ln)
        recs += sum(1 for x in v["alts"] if x != ".")
    return recs, time.perf_counter() - t0


def _cpu_c1_worker(k):
    """Reference-structured C1 path per record (oracle.c1_port_loop): metaseq id,
    short primary key, normalized alleles, end inference, cached bin lookup."""
    from oracle import avdb_oracle as O
    names, pos, refs, alts, exts = _SAMPLE[k]
    bi = O.PortBinIndex(_TABLE)
    t0 = time.perf_counter()
    n = O.c1_port_loop(names, pos, refs, alts, exts, bi)
    return n, time.perf_counter() - t0


def _cpu_c5_worker(k):
    """Reference-structured C5 path per record: end inference (VariantAnnotator),
    cached bin lookup (BinIndex), primary key (short join, or the VRS Allele digest
    through hashlib SHA-512 for long alleles), keep-first dedup on the key."""
    from oracle import avdb_oracle as O
    names, pos, refs, alts, exts, digs = _SAMPLE[k]
    bi = O.PortBinIndex(_TABLE)
    t0 = time.perf_counter()
    seen = set()
    for c, p, ref, alt, e in zip(names, pos, refs, alts, exts):
        end, _ = O.infer_end(p, ref, alt)
        try:
            bi.find_bin_index(c, p, end)
        except TypeError:  # unmappable (the GPU leg's status 2), as bin_index.py:75 raises
            pass
        dg = O.vrs_allele_digest(digs[c], p, ref, alt) if len(ref) + len(alt) > 50 else None
        pk = O.primary_key(c[3:] if c.startswith("chr") else c, p, ref, alt, e, digest=dg)
        if pk in seen:
            continue
        seen.add(pk)
    return len(pos), time.perf_counter() - t0


def _cpu_worker(k):
    from oracle import avdb_oracle as O
    names, pos, ends = _SAMPLE[k]
    bi = O.PortBinIndex(_TABLE)
    t0 = time.perf_counter()
    if ends is None:
        for c, p in zip(names, pos):
            bi.find_bin_index(c, p)
    else:
        for c, p, e in zip(names, pos, ends):
            bi.find_bin_index(c, p, e)
    return len(pos), time.perf_counter() - t0


def host_cpu_share():
    """``(cores, source)``: the host CPUs this process may use for the CPU baseline.
    A cgroup CPU quota (v2 ``cpu.max``, v1 ``cfs_quota_us``) is the share when one
    is set; else ``OMP_NUM_THREADS`` when it is below the affinity mask (the GPU
    box sets it to one GPU's CPU share while its affinity mask shows the whole
    machine); else ``len(os.sched_getaffinity(0))`` (BASELINE.md / SURVEY.md 8d)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and int(q) > 0:
            return max(1, min(aff, int(q) // int(per))), f"cgroup v2 cpu.max {q} {per} (affinity {aff})"
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, min(aff, q // per)), f"cgroup v1 cfs_quota_us {q} / cfs_period_us {per} (affinity {aff})"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), f"OMP_NUM_THREADS={omp}, no cgroup quota (affinity {aff})"
    return aff, "sched_getaffinity (no cgroup quota, no OMP_NUM_THREADS below it)"


def cpu_openmp(workload: str, threads: int, reps: int = 3):
    """the C oracle's per-record closed forms at -O3 with OpenMP on
    ``threads`` host threads (oracle/cpu_baseline.c) — a stronger comparator than the
    reference-structured port, on the same synthetic workload."""
    import ctypes
    import oracle
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.chromosomes import length_table
    lib = oracle.cpubase()
    lens = np.asarray(length_table(), dtype=np.uint32)
    P = lambda a: a.ctypes.data  # noqa: E731
    if workload in ("c2", "c3", "c4"):
        n = 20_000_000  # (a bounded sample: generating and sorting the whole set takes ~45 s)
        if workload == "c2":
            chrom, start = synth.np_point_snvs(n, seed=2)
            end = None
        else:
            chrom, start, end = synth.np_spans(n, seed=3 if workload == "c3" else 4, mix=workload)
        start = np.ascontiguousarray(start, dtype=np.uint32)
        end = None if end is None else np.ascontiguousarray(end, dtype=np.uint32)
        code = np.empty(n, np.uint32)
        st = np.empty(n, np.uint8)
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            lib.avdb_cpubase_bin_assign(P(chrom), P(start), None if end is None else P(end), n, P(lens), len(lens),
                                        P(code), P(st), threads)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return {"value": n / best, "unit": "variants/s", "cores": threads, "kind": "port-openmp",
                "sample": f"{n:,} records of the {workload.upper()} workload (numpy PCG64, sorted), the C oracle's closed "
                          f"form (oracle/cpu_baseline.c, gcc -O3 -fopenmp) on {threads} threads, best of {reps}: "
                          f"{best * 1e3:.1f} ms"}
    if workload in ("c4k", "c5"):
        n = 8_000_000 if workload == "c4k" else 4_000_000
        b = synth.dbsnp_alleles(n, seed=4, device="cpu") if workload == "c4k" else \
            synth.alleles(n, seed=5, device="cpu")
        h = {k: np.ascontiguousarray(getattr(b, k).numpy()) for k in ("chrom", "pos", "allele_off", "ref_len",
                                                                        "alt_len", "heap", "ext_id")}
        seqd = "".join("%032d" % i for i in range(25)).encode()
        end, code = np.empty(n, np.uint32), np.empty(n, np.uint32)
        st, keep = np.empty(n, np.uint8), np.empty(n, np.uint8)
        dig = np.empty(32 * n, np.uint8)
        mx = int(max(h["ref_len"].max(), h["alt_len"].max())) + 8
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            tb = lib.avdb_cpubase_keyed(P(h["chrom"]), P(h["pos"]), P(h["allele_off"]), P(h["ref_len"]),
                                        P(h["alt_len"]), P(h["heap"]), P(h["ext_id"]), n, P(lens), len(lens), 50,
                                        seqd, P(end), P(code), P(st), P(keep), P(dig), 65536, 2 * mx, threads)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return {"value": n / best, "unit": "variants/s", "cores": threads, "kind": "port-openmp",
                "sample": f"{n:,} {'dbSNP-mix' if workload == 'c4k' else 'ADSP-style'} records "
                          f"({workload.upper()} generator on the CPU); the C oracle's record prep + VRS digests + "
                          f"keys + ltree paths ({tb / n:.0f} B of text per record) + grouped dedup "
                          f"(oracle/cpu_baseline.c, gcc -O3 -fopenmp, chunks of 65,536 records) on {threads} "
                          f"threads, best of {reps}: {best * 1e3:.1f} ms"}
    return None


def cpu_baseline(workload: str, seconds_per_worker: float):
    """Reference-structured Python port (one-bin L13 cache + BinIndexRef table
    search on a miss, bin_index.py:59-75) over a bounded sample of the same
    workload, one process per host core like load_vcf_file.py:307-313; for the
    record workloads also the OpenMP comparator (``openmp``)."""
    try:
        host_cores = len(os.sched_getaffinity(0))
    except AttributeError:
        host_cores = os.cpu_count() or 1
    # one process per core of this process's CPU share (host_cpu_share: the cgroup
    # quota, else OMP_NUM_THREADS below the affinity mask, else the affinity mask)
    workers, core_source = host_cpu_share()
    res = _cpu_port(workload, seconds_per_worker, workers, host_cores)
    res["core_source"] = core_source
    if workload in ("c2", "c3", "c4", "c4k", "c5"):
        res["openmp"] = cpu_openmp(workload, workers)
        res["openmp"]["core_source"] = core_source
    return res


def _cpu_port(workload: str, seconds_per_worker: float, workers: int, host_cores: int):
    """The reference-structured Python port, ``workers`` processes."""
    global _SAMPLE, _TABLE
    import multiprocessing as mp
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.chromosomes import CHROM_NAMES, GRCH38_LENGTHS
    from oracle import avdb_oracle as O
    if workload == "c1":
        # the reference parallelises one process per chromosome file
        # (load_vcf_file.py:307-313): C1 is one file (chr22), so one process
        # over the whole C1 record set
        d = synth.np_c1(synth.C1_N, seed=1)
        heap = d["heap"].tobytes()
        o, r, a = d["allele_off"].tolist(), d["ref_len"].tolist(), d["alt_len"].tolist()
        _SAMPLE = [(["22"] * len(o), d["pos"].tolist(), [heap[x:x + y].decode() for x, y in zip(o, r)],
                    [heap[x + y:x + y + z].decode() for x, y, z in zip(o, r, a)],
                    ["rs%d" % e if e else None for e in d["ext_id"].tolist()])]
        _TABLE = O.BinTable(GRCH38_LENGTHS)
        n, t = _cpu_c1_worker(0)
        return {"value": n / t, "unit": "variants/s", "cores": 1, "workers": 1, "host_cores_visible": host_cores,
                "kind": "port",
                "per_core": n / t,
                "sample": f"the whole C1 set ({n:,} chr22 records), one process as the reference runs one "
                          f"chromosome file (load_vcf_file.py:307-313); oracle.c1_port_loop = the reference's "
                          f"per-record objects (an annotator per alt, the key from its metaseq id, normalized "
                          f"alleles, end inference on a second annotator) + PortBinIndex, {t:.2f} s",
                "calibration": {"port_over_reference_time": [0.85, 1.19],
                                "tool": "tools/calibrate_cpu_baseline.py calibrate_c1 (build container, the "
                                        "verbatim reference with the make_golden stub DB, same records)",
                                "log": "profiles/r06_calibrate_c1.txt",
                                "within_survey_8d_band": True}}
    if workload == "load":
        # ~80 us per line in the port (calibrated: 0.82x the verbatim reference's time)
        per = int(seconds_per_worker / 80e-6)
        lines = synth.vcf_text(per * workers, seed=6).decode().splitlines()
        _TABLE = O.BinTable(GRCH38_LENGTHS)
        _SAMPLE = [lines[k * per:(k + 1) * per] for k in range(workers)]
        ctx = mp.get_context("fork")
        t0 = time.perf_counter()
        with ctx.Pool(workers) as pool:
            res = pool.map(_cpu_load_worker, range(workers))
        wall = time.perf_counter() - t0
        n = sum(r[0] for r in res)
        return {"value": n / wall, "unit": "variants/s", "cores": workers, "workers": workers,
                "host_cores_visible": host_cores, "kind": "port",
                "sample": f"{per * workers:,} synthetic dbSNP-shaped VCF lines ({n:,} COPY rows), "
                          f"{workers} processes x {per:,} lines; reference-structured loader port "
                          f"(oracle/avdb_oracle.py load_line + PortBinIndex; 0.82x the verbatim "
                          f"reference's per-line time, tools/calibrate_cpu_baseline.py), per-process "
                          f"{np.mean([r[1] for r in res]):.2f} s"}
    if workload == "vcf":
        per = int(seconds_per_worker / 40e-6)  # ~40 us per line in the port
        lines = synth.vcf_text(per * workers, seed=6).decode().splitlines()
        _SAMPLE = [lines[k * per:(k + 1) * per] for k in range(workers)]
        ctx = mp.get_context("fork")
        t0 = time.perf_counter()
        with ctx.Pool(workers) as pool:
            res = pool.map(_cpu_vcf_worker, range(workers))
        wall = time.perf_counter() - t0
        n = sum(r[0] for r in res)
        return {"value": n / wall, "unit": "variants/s", "cores": workers, "workers": workers,
                "host_cores_visible": host_cores, "kind": "port",
                "sample": f"{per * workers:,} synthetic dbSNP-shaped VCF lines ({n:,} per-ALT records), "
                          f"{workers} processes x {per:,} lines; reference-structured VcfEntryParser parse + "
                          f"get_variant + per-ALT explode (oracle/avdb_oracle.py parse_vcf_line), per-process "
                          f"{np.mean([r[1] for r in res]):.2f} s"}
    if workload in ("c5", "c4k"):
        # ADSP-style (or dbSNP-mix) records generated on the CPU (same generator, CPU stream)
        per = int(seconds_per_worker / 6e-6)  # ~5.6 us per record in the port
        b = synth.alleles(per * workers, seed=5, device="cpu") if workload == "c5" else \
            synth.dbsnp_alleles(per * workers, seed=4, device="cpu")
        heap = b.heap.numpy().tobytes()
        off, rl, al = b.allele_off.numpy(), b.ref_len.numpy(), b.alt_len.numpy()
        names = [CHROM_NAMES[c] for c in b.chrom.numpy().tolist()]
        pos = b.pos.numpy().tolist()
        refs = [heap[o:o + r].decode() for o, r in zip(off.tolist(), rl.tolist())]
        alts = [heap[o + r:o + r + a].decode() for o, r, a in zip(off.tolist(), rl.tolist(), al.tolist())]
        exts = ["rs%d" % e if e else None for e in b.ext_id.numpy().tolist()]
        digs = {n: "%032d" % i for i, n in enumerate(CHROM_NAMES)}  # as the GPU leg's refget ids
        _TABLE = O.BinTable(GRCH38_LENGTHS)
        _SAMPLE = [(names[k * per:(k + 1) * per], pos[k * per:(k + 1) * per], refs[k * per:(k + 1) * per],
                    alts[k * per:(k + 1) * per], exts[k * per:(k + 1) * per], digs) for k in range(workers)]
        ctx = mp.get_context("fork")
        t0 = time.perf_counter()
        with ctx.Pool(workers) as pool:
            res = pool.map(_cpu_c5_worker, range(workers))
        wall = time.perf_counter() - t0
        n = sum(r[0] for r in res)
        return {"value": n / wall, "unit": "variants/s", "cores": workers, "workers": workers,
                "host_cores_visible": host_cores, "kind": "port",
                "sample": f"{n:,} {'ADSP-style' if workload == 'c5' else 'dbSNP-mix'} records "
                          f"({workload.upper()} generator on the CPU), {workers} processes x "
                          f"{per:,} records; reference-structured end inference + PortBinIndex + primary "
                          f"key (hashlib SHA-512 VRS digests for long alleles) + keep-first dedup "
                          f"(oracle/avdb_oracle.py), per-process {np.mean([r[1] for r in res]):.2f} s"}
    per = int(seconds_per_worker / 0.9e-6)  # ~0.9 us per cached find_bin_index call
    total = per * workers
    if workload == "c2":
        chrom, pos = synth.np_point_snvs(total, seed=2)
        end = None
    else:
        chrom, pos, end = synth.np_spans(total, seed=3 if workload == "c3" else 4, mix=workload)
    names = [CHROM_NAMES[c] for c in chrom.tolist()]
    pos = pos.tolist()
    end = end.tolist() if end is not None else None
    _TABLE = O.BinTable(GRCH38_LENGTHS)
    _SAMPLE = [(names[k * per:(k + 1) * per], pos[k * per:(k + 1) * per],
                end[k * per:(k + 1) * per] if end is not None else None) for k in range(workers)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, range(workers))
    wall = time.perf_counter() - t0
    n = sum(r[0] for r in res)
    return {"value": n / wall, "unit": "variants/s", "cores": workers, "workers": workers,
            "host_cores_visible": host_cores, "kind": "port",
            "sample": f"{n:,} records of the {workload.upper()} workload (numpy PCG64, sorted), "
                      f"{workers} processes x {per:,} records; reference-structured PortBinIndex "
                      f"(oracle/avdb_oracle.py), per-process {np.mean([r[1] for r in res]):.2f} s"}


# ---------------------------------------------------------------------------
def dropin(a):
    """Per-call latency of the drop-in API, called exactly as the reference's
    loader calls the reference API (one record / one line at a time)."""
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.bin_index import BinIndex
    from annotatedvdb_amd.loaders import VCFVariantLoader
    from annotatedvdb_amd.chromosomes import CHROM_NAMES, GRCH38_LENGTHS

    def per_call(fn, items, reps=1):
        fn(items[:20])  # warm (first launch, pinned buffers)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(items)
        return (time.perf_counter() - t0) / (reps * len(items)) * 1e6

    res = {}
    d = synth.np_c1(200_000, seed=1)
    # hits: sorted chr22 SNV/indel positions (vcf_variant_loader.py:310-311 pattern)
    bi = BinIndex(None, verbose=False)
    pos = d["pos"].tolist()
    res["find_bin_index_sorted_us"] = per_call(lambda xs: [bi.find_bin_index("22", p, p) for p in xs], pos)
    rng = np.random.default_rng(9)
    L = GRCH38_LENGTHS["22"]
    st = rng.integers(1, L - 1_100_000, 3000)
    sp = (10 ** rng.uniform(np.log10(16_000), 6, 3000)).astype(np.int64)
    spans = list(zip(st.tolist(), (st + sp).tolist()))
    bi2 = BinIndex(None, verbose=False)
    res["find_bin_index_miss_us"] = per_call(lambda xs: [bi2.find_bin_index("22", s, e) for s, e in xs], spans)
    lines = synth.vcf_text(3000, seed=17).decode().splitlines()

    def fresh():
        ld = VCFVariantLoader("dbSNP")
        ld.initialize_pk_generator("GRCh38", None)
        ld.initialize_bin_indexer(None)
        ld.set_algorithm_invocation_id(1)
        ld.initialize_copy_sql()
        return ld
    ld = fresh()
    res["parse_variant_per_line_us"] = per_call(lambda xs: [ld.parse_variant(x) for x in xs], lines)
    ld = fresh()
    res["parse_variants_batch_per_line_us"] = per_call(lambda xs: ld.parse_variants(xs), lines, reps=3)
    ld = fresh()
    text = ("\n".join(lines) + "\n").encode()
    res["load_vcf_text_per_line_us"] = per_call(lambda xs: ld.load_vcf_text(text if len(xs) > 20 else
                                                                            ("\n".join(xs) + "\n").encode()),
                                                lines, reps=3)
    # VariantAnnotator per alt allele, as vcf_parser.py:225-231 / vcf_variant_loader.py:309
    # construct and call it (one instance per call): K8a through the avdb_percall binding
    from annotatedvdb_amd.variant_annotator import VariantAnnotator
    heap = d["heap"].tobytes()
    o_, rl_, al_ = d["allele_off"].tolist(), d["ref_len"].tolist(), d["alt_len"].tolist()
    alle = [(heap[x:x + y].decode(), heap[x + y:x + y + z].decode(), p)
            for x, y, z, p in zip(o_[:50000], rl_[:50000], al_[:50000], pos[:50000])]
    res["annotator_end_us"] = per_call(
        lambda xs: [VariantAnnotator(r, a_, "22", p).infer_variant_end_location() for r, a_, p in xs], alle)
    res["annotator_normalized_us"] = per_call(
        lambda xs: [VariantAnnotator(r, a_, "22", p).get_normalized_alleles() for r, a_, p in xs], alle)
    res["annotator_display_us"] = per_call(
        lambda xs: [VariantAnnotator(r, a_, "22", p).get_display_attributes() for r, a_, p in xs], alle)
    res["per_line_path"] = {"k5h_rendered_lines": ld._engine.line_host().rendered,
                            "note": "parse_variant: K5h (avdb_vcf_line_host, the kernels' per-line code in the "
                                    "library's host code) for the lines it renders, else K8h (avdb_small_prep_host) "
                                    "or the general path; find_bin_index misses: K1h (avdb_bin_path_host)"}
    # the same calls through the reference-structured port on this host, same process,
    # same inputs (oracle.load_line: VcfEntryParser-style parse, per-alt VariantAnnotator-
    # style normalize + end, PortBinIndex with the reference's one-bin L13 cache and a
    # BinIndexRef table search on a miss, primary key, FREQ + display attributes, COPY
    # row and .mapping line; 0.82x the verbatim reference's per-line time in the build
    # container, tools/calibrate_cpu_baseline.py)
    from oracle import avdb_oracle as O
    from annotatedvdb_amd.chromosomes import length_table
    lens = length_table()
    pbi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    base = {"parse_variant_per_line_us": per_call(lambda xs: [O.load_line(x, lens, bin_index=pbi) for x in xs],
                                                  lines)}
    pbi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    base["find_bin_index_sorted_us"] = per_call(lambda xs: [pbi.find_bin_index("chr22", p, p) for p in xs], pos)
    pbi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    base["find_bin_index_miss_us"] = per_call(lambda xs: [pbi.find_bin_index("chr22", s, e) for s, e in xs],
                                              spans)
    PVA = O.PortVariantAnnotator
    base["annotator_end_us"] = per_call(
        lambda xs: [PVA(r, a_, "22", p).infer_variant_end_location() for r, a_, p in xs], alle)
    base["annotator_normalized_us"] = per_call(
        lambda xs: [PVA(r, a_, "22", p).get_normalized_alleles() for r, a_, p in xs], alle)
    base["annotator_display_us"] = per_call(
        lambda xs: [PVA(r, a_, "22", p).get_display_attributes() for r, a_, p in xs], alle)
    try:
        host_cores = len(os.sched_getaffinity(0))
    except AttributeError:
        host_cores = os.cpu_count() or 1
    cpu = {"value": base["parse_variant_per_line_us"], "unit": "us/line", "cores": 1, "workers": 1,
           "host_cores_visible": host_cores, "kind": "port", "per_call": base,
           "sample": "the same 3,000 dbSNP-shaped lines, 200,000 sorted chr22 positions and 3,000 > 15.6 kb spans, "
                     "one process on this host, per call as the reference's loader calls it (single-threaded per "
                     "process, load_vcf_file.py:307-313); the miss cost excludes the Postgres round trip the "
                     "reference pays (no database here)"}
    res["reference_build_container"] = {"parse_variant_per_line_us": 94.0, "find_bin_index_hit_us": 0.81,
                                        "find_bin_index_miss_us_fake_db": 8.2,
                                        "source": "SURVEY.md 6 / tools/calibrate_cpu_baseline.py (verbatim "
                                                  "reference with an in-process table-search DB, build container)"}
    res["vs_cpu_baseline"] = {k: base[k] / res[k] for k in ("parse_variant_per_line_us", "find_bin_index_sorted_us",
                                                             "find_bin_index_miss_us", "annotator_end_us",
                                                             "annotator_normalized_us", "annotator_display_us")}
    out = {"metric": "drop-in per-call latency (find_bin_index, parse_variant)", "value":
           res["parse_variant_per_line_us"], "unit": "us/line", "n_gpus": 1, "higher_is_better": False,
           "dtype": "u8", "data": "synthetic C1 records / dbSNP-shaped VCF lines", "config":
           {"workload": WORKLOADS["dropin"]["desc"]}, "latency": res, "cpu_baseline": cpu}
    print(json.dumps(out), flush=True)


def launch_command(a, port: int):
    """The torchrun command that starts ``--gpus`` ranks of this script (one
    process per GPU), as the driver's own N>1 form does."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]


def launch(a) -> int:
    """``bench.py --gpus N`` without torchrun's environment: start N ranks as a
    child torchrun (before this process touches the GPU — nothing is re-exec'd)
    and relay rank 0's JSON line; other output goes to stderr.  The reference's
    driver starts its own workers too (load_vcf_file.py:307-313)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    pr = subprocess.Popen(launch_command(a, port), stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    for line in pr.stdout:
        if line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return pr.wait()


def check_world(a, env=None) -> str:
    """'launch' (start --gpus ranks), 'run' (this process is a rank), or raise
    on a torchrun world that disagrees with --gpus."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if a.gpus > 1 else "run"
    if int(ws) != a.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {a.gpus}: launch N ranks with --gpus N")
    return "run"


def dry_run(a):
    """--dry-run: the N-rank plumbing alone (process group, all-gather, max over
    ranks, one JSON line from rank 0) with gloo on the CPU — the launcher's test."""
    from annotatedvdb_amd import distributed as D
    ri = D.init("gloo")
    ctr = torch.zeros(32, dtype=torch.int64)
    ctr[20] = 100
    ex = D.node_exchange(None, ri)  # (gloo: the torch.distributed exchange)
    _, node = ex.allgather(torch.zeros(8, dtype=torch.int32), ctr)
    t = D.max_over_ranks(0.001 * (1 + ri.rank), ri)
    if ri.rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": ri.world, "dry_run": True,
                          "ms_per_step": t * 1e3, "config": {"records_total": int(node[20].item()),
                                                              "exchange": ex.kind}}), flush=True)
    D.finalize(ri)


def main():
    a = parse()
    if a.workload == "dropin":
        torch.cuda.set_device(0)
        dropin(a)
        return
    if check_world(a) == "launch":
        sys.exit(launch(a))
    if a.dry_run:
        dry_run(a)
        return
    from annotatedvdb_amd import distributed as D
    ri = D.rank_info()
    # the north_star path rides along the default line: the keyed 1B-shard step (C4k)
    keyed = a.keyed == "on" or (a.keyed == "auto" and a.workload == "c2")
    # CPU baselines first, before this process touches the GPU (their worker
    # processes are forked and must not inherit an initialised HIP runtime)
    want_cpu = a.cpu_baseline == "on" or (a.cpu_baseline == "auto" and ri.world == 1
                                          and a.workload in ("c1", "c2", "c3", "c4", "c5", "c4k", "load", "vcf"))
    cpu = cpu_baseline(a.workload, a.cpu_seconds) if (ri.rank == 0 and want_cpu) else None
    cpu_k = cpu_baseline("c4k", a.cpu_seconds) if (keyed and ri.rank == 0 and want_cpu) else None
    ri = D.init("nccl")
    dev = torch.device("cuda", D.device_index(ri))
    torch.cuda.set_device(dev)
    out = run_workload(a, a.workload, ri, dev, cpu)
    if keyed:
        torch.cuda.empty_cache()
        k = run_workload(a, "c4k", ri, dev, cpu_k)
        out["keyed"] = {key: k[key] for key in ("metric", "value", "unit", "ms_per_step", "dtype", "config",
                                                "roofline", "k7_roofline", "cpu_baseline")}
        out["keyed"]["note"] = ("north_star's keyed path on BASELINE configs[3]'s per-GPU shard (1.25e8 of the "
                                "1e9 records): K2 end + bin, K3 dedup, K4 VRS digests, K7 primary-key + ltree-path "
                                "text; same steps / warmup, timed the same way")
    if ri.rank == 0:
        print(json.dumps(out), flush=True)
    D.finalize(ri)


def run_workload(a, name, ri, dev, cpu):
    """One workload on this rank's GPU: resident synthetic batch, warmup, K timed
    steps between barriers, max over ranks; returns the JSON object."""
    from annotatedvdb_amd import distributed as D
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.engine import Engine

    W = WORKLOADS[name]
    n = a.n or W["n"]
    pieces = D.my_pieces(ri)
    eng = Engine(dev.index)
    if name in ("c5", "c4k"):
        digs = ["%032d" % i for i in range(25)]  # synthetic refget ids (no SeqRepo offline)
        eng.set_sequence_digests(digs)

    # ---- resident synthetic batch (untimed) ----
    seed = 1000 * ri.rank
    if name == "c2":
        chrom, start = synth.point_snvs(n, seed=2 + seed, device=dev, pieces=pieces)
        end = None
    elif name in ("c3", "c4"):
        chrom, start, end = synth.spans(n, seed=(3 if name == "c3" else 4) + seed, device=dev,
                                        pieces=pieces, mix=name)
    elif name == "c1":
        batch = synth.c1_batch(n, seed=1, device=dev)
        heap_bytes = int(batch.heap.numel())
    elif name == "c4k":
        batch = synth.dbsnp_alleles(n, seed=4 + seed, device=dev, pieces=pieces)
        heap_bytes = int(batch.heap.numel())
    elif name in ("vcf", "load"):
        tile = synth.vcf_text(min(VCF_TILE, n), seed=6 + seed)
        reps = -(-n // min(VCF_TILE, n))
        text = torch.frombuffer(bytearray(tile), dtype=torch.uint8).to(dev).repeat(reps)
        n = reps * min(VCF_TILE, n)
        probe = eng.vcf_tokenize(text)
        n_rec = int(probe.records.n)
        heap_bytes = int(probe.records.heap.numel())
        del probe
    else:
        batch = synth.alleles(n, seed=5 + seed, device=dev, pieces=pieces)
        heap_bytes = int(batch.heap.numel())
    hist = eng.new_histogram()
    ctr = eng.new_counters()
    code = torch.empty(n, dtype=torch.int32, device=dev)
    # the job's exchange: the C ABI's RCCL all-gather (avdb_hist_allgather) when the
    # process group is RCCL, torch.distributed for the gloo rehearsal (D.node_exchange)
    try:
        ex = D.node_exchange(eng, ri)
    except Exception as e:  # (reported in the line, never silent: config.exchange)
        ex = D.TorchExchange(ri)
        ex.kind = "torch.distributed (C-ABI RCCL exchange failed to start: %s)" % (e,)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    evs = {}

    def timed(stage, record, fn, on=None):
        if not record:
            fn()
            return
        s_ = on if on is not None else stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s_)
        fn()
        e1.record(s_)
        evs.setdefault(stage, []).append((e0, e1))

    # C1 / C4k: the keyed record-prep step (annotatedvdb_amd.pipeline.KeyedStep, the
    # object the parity tests run), in the layouts pipeline.C1_LAYOUT / C4K_LAYOUT name
    # (C1: K2, K3, K7, no long records, captured as one HIP graph).  AVDB_BENCH_LAYOUT
    # (serial | fork: K3 on a second stream beside K7 | overlap: K7 beside K4 with the
    # digests filled afterwards) overrides either for an A/B; AVDB_BENCH_NARROW=0|1 the
    # layout's choice of u32 (AVDB_KEYS_OFF32) or u64 key / path offsets.
    ks = ps = None
    if name == "c5":
        from annotatedvdb_amd.pipeline import PrepStep
        ps = PrepStep(eng, batch, hist=hist, counters=ctr)
    if name in ("c1", "c4k"):
        from annotatedvdb_amd.pipeline import C1_LAYOUT, C4K_LAYOUT, KeyedStep
        layout = os.environ.get("AVDB_BENCH_LAYOUT", C1_LAYOUT if name == "c1" else C4K_LAYOUT)
        ks = KeyedStep(eng, batch, digests=name == "c4k", layout=layout, hist=hist, counters=ctr,
                       k4_grid=int(os.environ.get("AVDB_BENCH_K4_GRID", "0")),
                       k7_grid=int(os.environ.get("AVDB_BENCH_K7_GRID", "0")),
                       narrow_offsets={"1": True, "0": False}.get(os.environ.get("AVDB_BENCH_NARROW", "")))

    def step(record: bool):
        if ks is not None:
            # (stage events on the stream each stage ran on, and the whole step on the
            # launch stream: with a second stream the stages overlap, so their sum is
            # not the step's kernel time)
            ks.run(evs if record else None)
        elif name in ("c2", "c3", "c4"):
            timed("bin_assign", record, lambda: eng.bin_assign(
                chrom, start, end, want_status=False, hist=hist, counters=ctr, out_code=code))
        elif name == "vcf":
            # (records only: the public 80-byte line table is for the load path, K5)
            count_free = os.environ.get("AVDB_BENCH_VCF_COUNTED", "0") != "1"  # (A/B: the counted records path)
            timed("vcf_tokenize", record, lambda: eng.vcf_tokenize(text, want_lines=False, count_free=count_free))
        elif name == "load":
            box = {}
            timed("vcf_tokenize", record, lambda: box.setdefault("vb", eng.vcf_tokenize(text)))
            vb = box["vb"]
            timed("record_prep", record, lambda: box.setdefault(
                "prep", eng.record_prep(vb.records, want_lcp=False)))
            p_end, p_code, p_status, _ = box["prep"]
            fr = eng.vcf_format(vb, p_end, p_code, p_status, alg_id="1", events=evs if record else None)
            last["fr"] = fr
        else:  # C5: pipeline.PrepStep (K2 with K4's codes and K3's marks, K3 resolve, K4)
            ps.run(evs if record else None)

    last = {}
    # (AVDB_BENCH_STAGE_EVENTS=0: no stage-breakdown pass after the timed region)
    stage_events = os.environ.get("AVDB_BENCH_STAGE_EVENTS", "1") != "0"
    for _ in range(a.warmup):
        step(False)
    use_graph = a.graph == "on" or (a.graph == "auto" and name == "c1")
    graph = None
    if use_graph:
        # the step captured once as a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm) and
        # replayed: the same kernels on the same resident batch, without one host launch each
        # (C1's 1.1 M records take less GPU time than its launches do)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step(False)
        graph.replay()
        torch.cuda.synchronize()
    # the job-level collective once untimed, so any lazy RCCL setup for the
    # all-gather is not charged to the timed region
    ex.allgather(hist, ctr)
    hist.zero_()
    ctr.zero_()
    torch.cuda.synchronize()
    D.barrier(ri)
    torch.cuda.synchronize()
    # The timed region carries no per-stage events (an event pair around every launch
    # cost C2 8 us per 157 us step, profiles/c2_ab/r05_stage_events_ab.log): one pair
    # around the whole loop on the launch stream gives the average step on the device.
    loop0, loop1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    loop0.record(stream)
    for _ in range(a.steps):
        if graph is not None:
            graph.replay()
        else:
            step(False)
    loop1.record(stream)
    # job-level exchange: per-rank L8 histograms + counters (RCCL all-gather)
    node_hist, node_ctr = ex.allgather(hist, ctr)
    torch.cuda.synchronize()
    D.barrier(ri)
    torch.cuda.synchronize()
    elapsed = D.max_over_ranks(time.perf_counter() - t0, ri, device=dev)
    loop_ms = loop0.elapsed_time(loop1) / a.steps
    # the stage breakdown: the same steps again after the timed region, plain launches
    # with an event pair per stage on the stream it ran on
    if stage_events:
        for _ in range(a.steps):
            step(True)
        torch.cuda.synchronize()
    stage_ms = {k: float(np.mean([e0.elapsed_time(e1) for e0, e1 in v])) for k, v in evs.items()}
    stage_ms["timed_step_events"] = loop_ms
    if graph is not None:
        stage_ms["graph_replay"] = True
    # the roofline's kernel time: the one-kernel steps (C2/C3/C4) and the whole-step
    # workloads (C1, C4k, vcf) from the timed loop's own events; C5's K2 and the load
    # workload's K5 write pass from the stage breakdown
    kname = {"c5": "record_prep", "load": "format_write"}.get(name)
    kern_ms = stage_ms[kname] if kname else loop_ms
    if name in ("vcf", "load"):
        n_lines, n = n, n_rec  # the unit is emitted variant records (per-ALT rows)
    total_records = n * ri.world * a.steps
    value = total_records / elapsed

    if name == "c4k":
        # SURVEY.md §8d per-record bytes of the keyed record path (34 + rlen + alen + 24 per
        # long record) plus the key and ltree-path text K7 writes, over the four kernels' time
        kt = ks.kt
        rl, al = batch.ref_len.long(), batch.alt_len.long()
        n_long = int(((rl + al) > 50).sum().item())
        text = int(kt.key_offsets(n)[n].item()) + int(kt.path_offsets(n)[n].item())
        bytes_per_launch = 34 * n + int((rl + al).sum().item()) + 24 * n_long + text
        # K7 alone: SoA in (chrom 1 + pos 4 + allele_off 8 + ref_len 4 + alt_len 4 + ext_id 8 +
        # code 4 = 33 B), the allele bytes of short records, 32 digest chars per long record;
        # out key_off + path_off (8 + 8, or 4 + 4 with AVDB_KEYS_OFF32 — the u64 base per
        # 4,096 records is < 0.01 B a record) + state 1 and the text
        short = (rl + al) <= 50
        short_bytes = int((rl + al)[short].sum().item())
        k7_bytes = (34 + (8 if kt.off32 else 16)) * n + short_bytes + 32 * n_long + text
        # the one-pass keyed prep (layout "onepass", k_keyed_onepass): the SoA once (29 B),
        # the allele bytes of short records; out end 4 + code 4 + status 1 + keep 1 + K4 code 1
        # + key_off 8 + path_off 8 + state 1 and the text (long keys' 32 digest chars come later)
        op_bytes = 57 * n + short_bytes + text
        # SURVEY 8d's keyed-record bytes alone (no text): the verdict's frac_8d
        bytes_8d = 34 * n + int((rl + al).sum().item()) + 24 * n_long
        del rl, al, short
    elif name == "c1":
        # SURVEY.md §8d per-record bytes of the C5-style record path (in chrom 1 + pos 4 +
        # heap_off 8 + rlen 4 + alen 4 + rs 4, the allele bytes, out bin 4 + end 4 +
        # keep 1) plus the text K7 writes (keys + ltree paths)
        kt = ks.kt
        rl, al = batch.ref_len.long(), batch.alt_len.long()
        text = int(kt.key_offsets(n)[n].item()) + int(kt.path_offsets(n)[n].item())
        bytes_per_launch = 34 * n + int((rl + al).sum().item()) + text
    elif name == "c5":
        # K2 algorithmic bytes per record (the keyed form pipeline.PrepStep runs): in chrom 1 +
        # pos 4 + allele_off 8 + ref_len 4 + alt_len 4 + ext_id 8 (K3's mark phase), out end 4 +
        # code 4 + status 1 + keep 1 + K4's long code 1 (= 40 B), plus the allele bytes end
        # inference must read: through the first ref/alt mismatch (lcp + 1, capped at each
        # allele's length) for every non-SNV record.  The inversion test of equal-length
        # alleles may read further; that is not counted (a lower bound).
        _, _, _, lcp = eng.record_prep(batch, want_lcp=True)
        rl, al = batch.ref_len.long(), batch.alt_len.long()
        need = (torch.minimum(lcp.long() + 1, rl) + torch.minimum(lcp.long() + 1, al))
        need = torch.where((rl == 1) & (al == 1), torch.zeros_like(need), need)
        bytes_per_launch = n * 40 + int(need.sum().item())
        # the same bytes at the memory's granularity: every read is a 128-B request
        # (profiles/traffic_c5.json), and a long record's ref and alt starts lie in
        # different lines, so the floor for these reads is the distinct 128-B heap
        # lines holding the needed bytes, plus the SoA and the outputs
        off = batch.allele_off.long()
        lines = []
        for beg, ln in ((off, torch.minimum(lcp.long() + 1, rl)), (off + rl, torch.minimum(lcp.long() + 1, al))):
            keep = need > 0
            b0, b1 = beg[keep] // 128, (beg[keep] + ln[keep] - 1) // 128
            span = (b1 - b0 + 1)
            idx = torch.repeat_interleave(b0, span) + (
                torch.arange(int(span.sum().item()), device=b0.device) -
                torch.repeat_interleave(torch.cumsum(span, 0) - span, span))
            lines.append(idx)
        line_bytes = n * 40 + 128 * int(torch.unique(torch.cat(lines)).numel())
        del lcp, need, rl, al, off, lines
    elif name == "load":
        # K5 write pass: text read once + line table (80 B) + rec_off (8) + both offset
        # arrays (16) + line state (1) per line + end/code/status (9) per record, and
        # the COPY + .mapping text written
        fr = last["fr"]
        out_bytes = int(fr.copy.numel()) + int(fr.mapping.numel())
        bytes_per_launch = int(text.numel()) + 105 * n_lines + 9 * n + out_bytes
    elif name == "vcf":
        # text read once + record SoA written (chrom 1, pos 4, allele_off 8, ref_len 4,
        # alt_len 4, ext_id 8, rec_line 4, rec_alt 4 = 37 B) + allele heap written
        bytes_per_launch = int(text.numel()) + 37 * n + heap_bytes
    else:
        bytes_per_launch = n * W["bytes_per"]
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "variants/s",
        "n_gpus": ri.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded GRCh38-shaped records generated on device)",
        "config": {"workload": W["desc"], "records_per_gpu": n, "records_total": n * ri.world,
                   "parallelism": f"dp{ri.world} (length-balanced 64 Mb genome pieces per rank)",
                   "records_processed": int(node_ctr[20].item()) // max(1, a.steps),
                   "exchange": ex.kind if ri.distributed or not isinstance(ex, D.TorchExchange) else None,
                   "stage_ms": stage_ms},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": W["kernel"], "kernel_ms": kern_ms,
                     "algorithmic_bytes_per_launch": bytes_per_launch},
        "cpu_baseline": cpu,
    }
    if name == "c5":
        out["roofline"]["line_granular"] = {
            "bytes_per_launch": line_bytes, "achieved": line_bytes / (kern_ms * 1e-3) / 1e9,
            "frac": line_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "note": "SoA + outputs + the distinct 128-B heap lines holding the bytes end inference needs "
                    "(the smallest read the memory serves); traffic / this = HBM bytes over the line floor"}
        # SURVEY.md 8d whole-pipeline bytes (34 + rlen + alen + 24 per long record) over
        # K2 + K3 + K4 time, and K4's VALU roofline (compute-bound SHA-512)
        rl, al = batch.ref_len.long(), batch.alt_len.long()
        n_long = int(((rl + al) > 50).sum().item())
        pipe_bytes = 34 * n + int((rl + al).sum().item()) + 24 * n_long
        pipe_ms = sum(stage_ms[k] for k in ("record_prep", "pk_dedup", "vrs_digest"))
        pipe = pipe_bytes / (pipe_ms * 1e-3) / 1e9
        out["pipeline_roofline"] = {"bound": "hbm", "achieved": pipe, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": pipe / HBM_PEAK_GBS, "algorithmic_bytes_per_step": pipe_bytes,
                                    "step_kernel_ms": pipe_ms,
                                    "note": "SURVEY 8d C5 bytes (34 + rlen + alen + 24 if long per record) / "
                                            "(K2 + K3 + K4 HIP-event time); K4 is VALU-bound, not HBM-bound"}
        k4 = os.path.join(ROOT, "profiles", "pmc_k4.json")
        if os.path.exists(k4):
            pk = json.load(open(k4))
            vi = float(pk["sq_insts_valu_per_launch"])
            ach = vi / (stage_ms["vrs_digest"] * 1e-3)
            peak = 1024 * 2.4e9 / 2  # one wave64 VALU instruction per 2 cycles per SIMD (157 TF fp32 basis)
            vop3 = 1024 * 2.4e9 / pk["vop3_cycles_per_wave_instr"]
            out["valu_roofline"] = {"kernel": "avdb_vrs_digest (k_long_hist/scan/scatter + k_vrs_digest)",
                                    "bound": "valu", "achieved": ach, "peak": peak, "unit": "wave-instr/s",
                                    "frac": ach / peak, "frac_of_vop3_issue_peak": ach / vop3,
                                    "vop3_issue_peak": vop3, "sq_insts_valu_per_launch": vi,
                                    "sha512_compressions_per_launch": pk.get("sha512_compressions_per_launch"),
                                    "note": pk.get("note")}
    if name == "c4k":
        kt = ks.kt
        out["dtype"] = "u8"
        out["data"] = "synthetic dbSNP-mix records (synth.dbsnp_alleles, torch PCG on device), resident in HBM"
        out["config"].update(key_bytes=int(kt.key_offsets(n)[n].item()), path_bytes=int(kt.path_offsets(n)[n].item()),
                             long_records=n_long, heap_bytes=heap_bytes,
                             duplicates=int(node_ctr[21].item()) // max(1, a.steps))
        out["config"]["layout"] = ks.layout
        out["roofline"]["frac_8d"] = bytes_8d / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
        out["roofline"]["algorithmic_bytes_8d"] = bytes_8d
        if ks.layout == "onepass":
            k7_ms = stage_ms["keyed_prep"]
            out["k7_roofline"] = {"kernel": "avdb_keyed_prep (k_keyed_onepass: K2 + K7 in one pass over the SoA, "
                                            "decoupled look-back over 256-record groups; + init and stats launches)",
                                  "bound": "hbm", "achieved": op_bytes / (k7_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": op_bytes / (k7_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                  "algorithmic_bytes_per_launch": op_bytes, "stage_ms": k7_ms}
            sc = stream_ceiling("read1_write3", os.path.join(ROOT, "profiles", "pmc_keyed_onepass.json"), k7_ms)
        else:
            k7_ms = stage_ms["primary_keys"]
            out["k7_roofline"] = {"kernel": "avdb_primary_keys_onepass_ex (group scan + LDS-staged write pass; "
                                            "group totals from the keyed K2)",
                                  "bound": "hbm", "achieved": k7_bytes / (k7_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": k7_bytes / (k7_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                  "algorithmic_bytes_per_launch": k7_bytes, "stage_ms": k7_ms}
            sc = stream_ceiling("read1_write3", os.path.join(ROOT, "profiles", "pmc_k7.json"), k7_ms)
        if sc:
            out["k7_roofline"]["stream_ceiling"] = sc
        out["roofline"]["note"] = ("achieved = SURVEY 8d keyed-record bytes (34 + rlen + alen + 24 if long) + "
                                   "key/path text written, over the timed loop's HIP-event time per step on the "
                                   "launch stream (" +
                                   {"onepass": "K2 + K7 as one pass (avdb_keyed_prep), then K3, K4 and the digest "
                                               "fill, in one stream",
                                    "serial": "K2 + K3 + K4 + K7 in one stream",
                                    "fork": "K2, then K4 + K7 with K3 beside them on a second stream, joined",
                                    "overlap": "K2, then K7 with the long keys' digests pending beside K4 + K3 on a "
                                               "second stream, joined, then the digest fill"}[ks.layout] +
                                   "); K4 (SHA-512) is VALU-bound, the others HBM-bound; stage_ms from an untimed "
                                   "pass with an event pair per stage")
    if name == "c1":
        kt = ks.kt
        out["dtype"] = "u8"
        out["data"] = "synthetic C1 records (numpy PCG64 seed 1, synth.np_c1), resident in HBM"
        out["config"].update(key_bytes=int(kt.key_offsets(n)[n].item()), path_bytes=int(kt.path_offsets(n)[n].item()),
                             duplicates=int(node_ctr[21].item()) // max(1, a.steps))
        out["roofline"]["note"] = ("achieved = SURVEY 8d record bytes + key/path text written / whole step "
                                   "time; at 1.1 M records the step is launch-bound (4 kernels in one HIP graph" +
                                   (", K3 on a parallel branch beside K7" if ks.layout == "fork" else "") +
                                   "), not HBM-bound")
        if cpu:
            out["cpu_baseline"]["reference_survey_per_core"] = "285-306 K variants/s (SURVEY.md 6, build container)"
    if name == "load":
        fr = last["fr"]
        out["dtype"] = "u8"
        out["data"] = "synthetic dbSNP-shaped VCF text with INFO FREQ (numpy PCG64 lines tiled on the device)"
        out["config"].update(host_lines=int(fr.counters[27].item()), lines_per_gpu=n_lines, text_bytes_per_gpu=int(text.numel()),
                             copy_bytes_per_gpu=int(fr.copy.numel()), mapping_bytes_per_gpu=int(fr.mapping.numel()),
                             records_processed=None)
        out["roofline"]["note"] = ("achieved = K5 write-pass algorithmic bytes (text + line table + offsets "
                                   "+ per-record inputs + COPY/.mapping text written) / its HIP-event time")
    if name == "vcf":
        out["dtype"] = "u8"
        out["data"] = "synthetic dbSNP-shaped VCF text (numpy PCG64 lines tiled on the device)"
        out["config"].update(lines_per_gpu=n_lines, text_bytes_per_gpu=int(text.numel()),
                             records_processed=None)
        out["roofline"]["note"] = ("achieved = algorithmic bytes / whole tokenize step, records only "
                                   "(vcf_tokenize(want_lines=False), the count-free path: window parse into "
                                   "window-local line slots, two window-total scans, one host read, per-window "
                                   "emit; AVDB_BENCH_VCF_COUNTED=1: count pass, parse, paired per-line scan, emit); "
                                   "the 16 B of line offsets per line it writes are not counted")
        out["config"]["path"] = {"local": "count-free", "counted": "counted"}.get(eng.last_vcf_path, eng.last_vcf_path)
    ex.close()
    return out




if __name__ == "__main__":
    main()
