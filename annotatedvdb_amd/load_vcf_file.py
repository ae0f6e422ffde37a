"""Multi-GPU load driver — the counterpart of ``Load/bin/load_vcf_file.py``.

The reference runs one OS process per chromosome file
(``load_vcf_file.py:307-313``, ``ProcessPoolExecutor(maxWorkers)``), each doing
the per-line loop of ``load()`` (:80-221): ``parse_variant`` per line, the
``.mapping`` line printed per line (:116-117), a COPY into Postgres every
``--commitAfter`` lines (:135-171).  Here one process per GPU (``torchrun``):

* several files (``--dir``/``--extension``/``--chr``): files are dealt to the
  ranks by size (LPT), each rank loads its files whole, as the reference's
  workers do;
* one file (``--fileName``) on N ranks: every rank streams the file in
  ``--batchBytes`` blocks, tokenizes each on its GPU (K0) and keeps the lines
  the genome-piece plan gives it (K9
  ``avdb_vcf_select_lines`` / ``_copy``: contigs cut at 64 Mb, pieces by LPT,
  ``shard.plan``); bins and keys need nothing from other ranks.

Each rank then runs the whole-batch GPU path (``VCFVariantLoader.load_vcf_text``:
K0 → K2 → K4 → K3 → K6 → K5) on batches of ``--batchBytes`` cut at line
boundaries and writes ``<out>/<file>.r<rank>.copy`` (the COPY rows the
reference streams into Postgres: there is no database here) and
``<out>/<file>.r<rank>.mapping``.  The only collective is one all-gather of the
per-rank counters at the end (RCCL on GPUs; gloo for CPU-side tests).

    torchrun --nproc-per-node 8 -m annotatedvdb_amd.load_vcf_file --fileName x.vcf --outDir out
    python -m annotatedvdb_amd.load_vcf_file --dir vcfs --extension vcf --chr all --outDir out
"""

from __future__ import annotations

import argparse
import gzip
import json
import logging
import os
import sys
import time
from typing import Dict, List, Optional, Sequence

LOGGER = logging.getLogger("load_vcf_file")
COUNTERS = ("line", "variant", "skipped", "duplicates", "update")


def parse_args(argv: Optional[Sequence[str]] = None):
    ap = argparse.ArgumentParser(allow_abbrev=False, description="load AnnotatedVDB COPY rows from VCF files "
                                 "on the GPUs of one node (one process per GPU)")
    ap.add_argument("-d", "--dir", help="directory containing chr<N>.<extension> files")
    ap.add_argument("-e", "--extension", help="file extension (e.g. vcf or vcf.gz)")
    ap.add_argument("-c", "--chr", help="comma separated chromosomes, or all / allNoM")
    ap.add_argument("--fileName", help="one VCF file (split over the ranks by genome pieces)")
    ap.add_argument("-g", "--genomeBuild", default="GRCh38")
    ap.add_argument("-s", "--seqrepoProxyPath", default=None,
                    help="chrom<TAB>refget-digest (or JSON) file for long-allele keys")
    ap.add_argument("--datasource", default="dbSNP",
                    choices=["dbSNP", "DBSNP", "dbsnp", "ADSP", "ADSP-FunGen", "NIAGADS", "EVA"])
    ap.add_argument("-m", "--chromosomeMap", help="tab-delimited source_id -> chromosome map (e.g. RefSeq "
                    "accessions used as CHROM), parsers.ChromosomeMap")
    ap.add_argument("--skipExisting", action="store_true")
    ap.add_argument("--existing", help="export of AnnotatedVDB.Variant: metaseq_id<TAB>record_primary_key<TAB>bin_index")
    ap.add_argument("--algInvocationId", default="0", help="row_algorithm_id of the COPY rows")
    ap.add_argument("--dedup", action="store_true", help="drop in-batch duplicate primary keys (keep first)")
    ap.add_argument("--batchBytes", type=int, default=256 << 20)
    ap.add_argument("--outDir", default=".")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl on GPUs)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args(argv)


def input_files(args) -> List[str]:
    if args.fileName:
        return [args.fileName]
    from .chromosomes import CHROM_NAMES
    chrs = CHROM_NAMES if (args.chr or "all").startswith("all") else args.chr.split(",")
    if args.chr == "allNoM":
        chrs = [c for c in chrs if c != "M"]
    return [os.path.join(args.dir, "chr%s.%s" % (c, args.extension)) for c in chrs]


def assign_files(files: List[str], world: int) -> List[List[str]]:
    """LPT over file sizes (the reference's pool takes files in list order)."""
    sizes = [(os.path.getsize(f) if os.path.exists(f) else 0, i) for i, f in enumerate(files)]
    load = [0] * world
    out: List[List[str]] = [[] for _ in range(world)]
    for sz, i in sorted(sizes, key=lambda x: (-x[0], x[1])):
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(files[i])
        load[r] += sz
    for r in range(world):
        out[r].sort(key=files.index)
    return out


def read_text(path: str) -> bytes:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as fh:
        return fh.read()


def iter_batches(path: str, batch_bytes: int):
    """The file as consecutive blocks of about ``batch_bytes`` cut after a newline
    (a line longer than a block stays whole): host memory stays bounded by the
    batch, whatever the file size (gzip streams too)."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as fh:
        carry = b""
        while True:
            block = fh.read(max(1, batch_bytes))
            if not block:
                break
            buf = carry + block
            k = buf.rfind(b"\n")
            if k < 0:
                carry = buf
                continue
            carry = buf[k + 1:]
            yield buf[:k + 1]
        if carry:
            yield carry


def make_loader(args, device: int):
    from .loaders import VCFVariantLoader
    ld = VCFVariantLoader(args.datasource, verbose=args.verbose, device=device)
    ld.initialize_pk_generator(args.genomeBuild, args.seqrepoProxyPath)
    ld.initialize_bin_indexer(None)
    ld.set_algorithm_invocation_id(args.algInvocationId)
    ld.initialize_copy_sql()
    if args.chromosomeMap:
        from .parsers import ChromosomeMap
        ld.set_chromosome_map(ChromosomeMap(args.chromosomeMap))
    if args.skipExisting:
        from .existing import ExistingVariants
        ld.set_skip_existing(True, existing=ExistingVariants.from_tsv(args.existing, engine=ld._engine))
    return ld


def rank_text(raw: bytes, loader, plan, rank: int) -> bytes:
    """The lines of ``raw`` the piece plan gives to ``rank`` (K0 + K9 on the GPU)."""
    eng = loader._engine
    vo = loader._gpu_vcf_opts()  # chromosome map: lines are placed by their mapped contig
    vb = eng.vcf_tokenize(raw, vo if isinstance(vo, type(eng.vcf_opts())) else None)
    return eng.vcf_select(vb, plan, rank).cpu().numpy().tobytes()


def load(path: str, args, loader, rank: int, plan=None) -> Dict[str, int]:
    """One input file (or this rank's share of it) through the GPU load path,
    streamed in ``--batchBytes`` blocks cut at line boundaries.  With a piece
    plan (one file on N ranks) every block is tokenized on this rank's GPU and
    only the lines its pieces own are kept (K0 + K9): a line's owner depends on
    the line alone, so block-wise selection equals whole-file selection."""
    base = os.path.join(args.outDir, os.path.basename(path))
    before = {k: loader.get_count(k) for k in COUNTERS}
    t0 = time.perf_counter()
    with open(base + ".r%d.mapping" % rank, "w") as mfh, open(base + ".r%d.copy" % rank, "w") as cfh:
        for block in iter_batches(path, args.batchBytes):
            if plan is not None:
                block = rank_text(block, loader, plan, rank)
                if not block:
                    continue
            loader.reset_copy_buffer()
            try:
                loader.load_vcf_text(block, dedup=args.dedup, mapping_out=mfh, batch_bytes=args.batchBytes)
            finally:
                cfh.write(loader.copy_buffer().getvalue())  # the rows the reference would COPY (:135-142)
        if loader.is_adsp():
            with open(base + ".r%d.updates" % rank, "w") as ufh:
                for pk, chrom in loader.update_buffer():
                    ufh.write("%s\t%s\n" % (pk, chrom))
            loader.reset_update_buffer()
    stats = {k: loader.get_count(k) - before[k] for k in COUNTERS}
    LOGGER.info("rank %d: %s -> %s (%.2f s) %s", rank, path, base, time.perf_counter() - t0, stats)
    return stats


def main(argv: Optional[Sequence[str]] = None) -> Dict[str, int]:
    args = parse_args(argv)
    logging.basicConfig(format="%(asctime)s %(levelname)-8s %(message)s", level=logging.INFO)
    import torch
    from . import distributed as D
    from . import shard
    ri = D.init(args.backend)
    device = ri.local if torch.cuda.device_count() > ri.local else 0
    torch.cuda.set_device(device)
    os.makedirs(args.outDir, exist_ok=True)
    loader = make_loader(args, device)
    files = input_files(args)
    totals = {k: 0 for k in COUNTERS}
    if args.fileName and ri.world > 1:
        plan = shard.plan(ri.world, loader._engine.lengths)
        mine = [(args.fileName, plan)]
    else:
        mine = [(f, None) for f in assign_files(files, ri.world)[ri.rank]]
    failed = 0
    for f, plan in mine:
        if not os.path.exists(f):
            LOGGER.info("Input file %s not found.  SKIPPING.", f)
            continue
        before = {k: loader.get_count(k) for k in COUNTERS}
        try:
            st = load(f, args, loader, ri.rank, plan)
        except Exception as err:  # noqa: BLE001 — a file fails alone, as a reference pool worker does
            # (load_vcf_file.py:212-214: logged critical, that file stops); the other files
            # and ranks go on, and the failure travels in the all-gathered counters
            LOGGER.critical("rank %d: problem parsing %s at variant %s: %r", ri.rank, f,
                            loader.get_current_variant_id(), err)
            failed += 1
            st = {k: loader.get_count(k) - before[k] for k in COUNTERS}
        for k in COUNTERS:
            totals[k] += st[k]
    # node totals: one all-gather of the per-rank counters (+ failed files), reached
    # by every rank whatever happened to its files, so no rank waits on a dead peer
    mine_t = torch.tensor([totals[k] for k in COUNTERS] + [failed], dtype=torch.int64,
                          device="cuda" if (args.backend or "nccl") == "nccl" and ri.distributed else "cpu")
    if ri.distributed:
        import torch.distributed as dist
        parts = [torch.empty_like(mine_t) for _ in range(ri.world)]
        dist.all_gather(parts, mine_t)
        node = torch.stack(parts).sum(0).cpu().tolist()
    else:
        node = mine_t.cpu().tolist()
    node_totals = dict(zip(COUNTERS, node[:len(COUNTERS)]))
    node_failed = int(node[len(COUNTERS)])
    if ri.rank == 0:
        LOGGER.info("node totals: %s; failed files: %d", node_totals, node_failed)
        print(json.dumps({"node_totals": node_totals, "failed_files": node_failed, "ranks": ri.world}), flush=True)
    D.finalize(ri)
    if node_failed:
        raise LoadFailed("%d input file(s) failed on the node (this rank: %d); see the CRITICAL log lines"
                         % (node_failed, failed))
    return node_totals


class LoadFailed(RuntimeError):
    """At least one rank could not load one of its files (every rank raises it
    after the node-wide counter exchange, so the job exits non-zero)."""


if __name__ == "__main__":
    main(sys.argv[1:])
