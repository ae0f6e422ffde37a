"""The keyed record-prep step over one resident batch, as one object: what
``bench.py`` times for C1 and C4k (BASELINE configs[0] and the per-GPU shard of
configs[3]) and what ``tests/test_gpu_c4k.py`` / ``tests/test_gpu_c1.py`` check
against the C oracle — the same calls, buffers and stream layout, so the benched
form is the checked form.

One step (north_star's "bin path plus primary-key generation and dedup before the
DB write"; Load/lib ``VCFVariantLoader.__parse_alt_alleles``,
vcf_variant_loader.py:259-348, batched):

  K2  avdb_record_prep_keyed       end, bin code, status (variant_annotator.py:36-79,
                                   bin_index.py:59-75); it also writes K7's group totals,
                                   K4's long-record codes and K3's first phase
  K3  avdb_pk_dedup_ex (MARKED)    keep-first per primary key (removeDuplicates.sql:2-24)
  K4  avdb_vrs_digest_ex           VRS digests of the long records (primary_key_generator.py:125-165)
  K7  avdb_primary_keys_onepass_ex keys + ltree paths as text (primary_key_generator.py:99-122)

Layouts (``layout``):
  ``onepass``  K2 and K7 as ONE pass over the SoA (avdb_keyed_prep: K2's outputs,
               K3's marks, K4's codes and the keys + paths with the long keys'
               digests pending; text offsets by a decoupled look-back over
               1,024-record groups), then K3, then K4, which also writes the
               digests into the pending keys (avdb_vrs_digest_keys);
  ``serial``   K2, K3, K4, K7 in the launch stream;
  ``fork``     K3 on a second stream beside K4 / K7 (it reads only K2's outputs and
               nothing reads keep until the step ends), joined at the end;
  ``overlap``  K7 does not wait for K4: it lays out the long keys with their digest
               characters pending (AVDB_KEYS_DIGEST_DEFERRED) while K4 (SHA-512,
               VALU-bound) runs on a second stream beside the store-bound K7, then
               K3 follows K4 there, and the step joins and fills the digests
               (avdb_primary_keys_fill_digests).

All buffers the kernels hand each other (the K7 workspace and text buffers, the
K3 and K4 workspaces) are allocated once, in ``__init__``; the per-step outputs
(end / code / status, keep, digests) come from the engine per call, as in any
caller's loop.
"""

from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from . import _native as N

LAYOUTS = ("onepass", "serial", "fork", "overlap")
# what bench.py times for C4k (AVDB_BENCH_LAYOUT overrides there) and what
# tests/test_gpu_c4k.py checks over the whole 1e9-record job
C4K_LAYOUT = "serial"
# what bench.py times for C1 (captured as one HIP graph) and what
# tests/test_gpu_c1.py replays: on this round's boxes the graph with K3 on a
# parallel branch replays slower than the one-stream graph (0.112 vs 0.097 ms per
# step; plain launches of the fork 0.099 ms), profiles/c1_ab/r05_layout_graph_ab.log
C1_LAYOUT = "serial"


def _timed(events, name, stream, fn):
    """fn() with an event pair around it on ``stream`` (``events[name]``), or plain."""
    if events is None:
        return fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    r = fn()
    e1.record(stream)
    events.setdefault(name, []).append((e0, e1))
    return r


class KeyedStep:
    def __init__(self, engine, batch, *, digests: bool, layout: str = "serial", max_seq_len: int = 50,
                 hist: Optional[torch.Tensor] = None, counters: Optional[torch.Tensor] = None,
                 k4_grid: int = 0, k7_grid: int = 0, narrow_offsets: Optional[bool] = None):
        if layout not in LAYOUTS:
            raise ValueError("layout must be one of %s" % (LAYOUTS,))
        if layout == "overlap" and not digests:
            raise ValueError("the overlap layout runs K4 beside K7: it needs digests")
        self.eng, self.b = engine, batch
        self.digests, self.layout, self.max_seq_len = bool(digests), layout, int(max_seq_len)
        self.hist, self.counters = hist, counters
        n = batch.n
        dev = engine.device
        # the key / path offsets in the narrow layout (AVDB_KEYS_OFF32: 4 bytes per record and
        # stream instead of 8) where no later stage of the step reads them as u64 (the
        # overlap layout's digest fill and the one-pass prep do)
        if narrow_offsets is None:
            narrow_offsets = layout in ("serial", "fork")
        self.kt = engine.new_key_text(n, int(batch.heap.numel()), paths=True, off32=bool(narrow_offsets))
        # K3 list workspace (+ 2^22 entries: the keyed K2's per-workgroup suspect slices round up)
        self.ws3 = engine.empty(16384 + 4 * (((n + 3) & ~3) + (1 << 22)), torch.uint8)
        self.ws4 = None
        if self.digests:
            sz = ctypes.c_size_t()
            engine.lib.avdb_vrs_digest_workspace_size(n, ctypes.byref(sz))
            self.ws4 = engine.empty(int(sz.value), torch.uint8)
        # both grid options every time (0 = the library's default), so a capped grid
        # from an earlier step on this engine never carries over
        engine.set_option(N.OPT_K4_GRID, int(k4_grid))
        engine.set_option(N.OPT_K7_GRID, int(k7_grid))
        self.ws_op = None
        if layout == "onepass":
            sz = ctypes.c_size_t()
            engine.lib.avdb_keyed_prep_workspace_size(n, ctypes.byref(sz))
            self.ws_op = engine.empty(int(sz.value), torch.uint8)
        self.side = torch.cuda.Stream(dev) if layout in ("fork", "overlap") else None
        self.out: Dict[str, object] = {}

    # ---- one step ----------------------------------------------------------
    def _timed(self, events, name, stream, fn):
        return _timed(events, name, stream, fn)

    def run(self, events: Optional[dict] = None) -> Dict[str, object]:
        """One step on the current stream; returns (and keeps in ``self.out``)
        ``end, code, status, keep, digest, is_long, kt``.  ``events``: per-stage
        HIP event pairs (on the stream each stage ran on) and ``step_span`` on the
        launch stream."""
        eng, b, kt, msl = self.eng, self.b, self.kt, self.max_seq_len
        main = torch.cuda.current_stream(eng.device)
        side = self.side
        t = lambda name, s, fn: self._timed(events, name, s, fn)  # noqa: E731
        span0 = None
        if events is not None:
            span0 = torch.cuda.Event(enable_timing=True)
            span0.record(main)
        dedup = lambda: eng.pk_dedup(b, grouped=True, counters=self.counters, workspace=self.ws3)  # noqa: E731
        digest = lambda: eng.vrs_digest(b, msl, workspace=self.ws4)  # noqa: E731
        dig = is_long = keep = None
        if self.layout == "onepass":
            end, code, status, _ = t("keyed_prep", main, lambda: eng.keyed_prep(
                b, kt, max_seq_len=msl, defer_digest=self.digests, hist=self.hist, counters=self.counters,
                digest_workspace=self.ws4, dedup_workspace=self.ws3, workspace=self.ws_op))
            keep = t("pk_dedup", main, dedup)
            if self.digests:  # (K4 writes the pending keys' digest characters too)
                dig, is_long = t("vrs_digest", main, lambda: eng.vrs_digest(b, msl, workspace=self.ws4, keys=kt))
            if events is not None:
                span1 = torch.cuda.Event(enable_timing=True)
                span1.record(main)
                events.setdefault("step_span", []).append((span0, span1))
            self.out = dict(end=end, code=code, status=status, keep=keep, digest=dig, is_long=is_long, kt=kt)
            return self.out
        end, code, status, _ = t("record_prep", main, lambda: eng.record_prep(
            b, want_lcp=False, hist=self.hist, counters=self.counters, keys=kt, key_digest=self.digests,
            max_seq_len=msl, digest_workspace=self.ws4, dedup_workspace=self.ws3))
        if self.layout == "serial":
            keep = t("pk_dedup", main, dedup)
            if self.digests:
                dig, is_long = t("vrs_digest", main, digest)
            t("primary_keys", main, lambda: eng.primary_keys(b, code=code, digest=dig, max_seq_len=msl, out=kt))
        elif self.layout == "fork":
            side.wait_stream(main)
            with torch.cuda.stream(side):
                keep = t("pk_dedup", side, dedup)
            if self.digests:
                dig, is_long = t("vrs_digest", main, digest)
            t("primary_keys", main, lambda: eng.primary_keys(b, code=code, digest=dig, max_seq_len=msl, out=kt))
            main.wait_stream(side)
            keep.record_stream(main)
        else:  # overlap
            side.wait_stream(main)
            with torch.cuda.stream(side):
                dig, is_long = t("vrs_digest", side, digest)
                keep = t("pk_dedup", side, dedup)
            t("primary_keys", main, lambda: eng.primary_keys(b, code=code, max_seq_len=msl, out=kt,
                                                             defer_digest=True))
            main.wait_stream(side)
            for x in (dig, is_long, keep):
                x.record_stream(main)
            t("fill_digests", main, lambda: eng.fill_digests(b, dig, kt))
        if events is not None:
            span1 = torch.cuda.Event(enable_timing=True)
            span1.record(main)
            events.setdefault("step_span", []).append((span0, span1))
        self.out = dict(end=end, code=code, status=status, keep=keep, digest=dig, is_long=is_long, kt=kt)
        return self.out


class PrepStep:
    """The keyed record-prep step without key text (BASELINE configs[4], C5: "bin path +
    hashed primary key + dedup"): K2 (end, bin, status) also classifying the long
    records for K4 and running K3's first phase (``avdb_record_prep_keyed`` with no K7
    workspace), K3 resolving only the listed runs, K4 from K2's codes — what
    ``bench.py --workload c5`` times and ``tests/test_gpu_parity.py`` checks against
    the C oracle over the whole 2e8-record job.  Workspaces are allocated once."""

    def __init__(self, engine, batch, *, max_seq_len: int = 50, hist: Optional[torch.Tensor] = None,
                 counters: Optional[torch.Tensor] = None):
        self.eng, self.b, self.max_seq_len = engine, batch, int(max_seq_len)
        self.hist, self.counters = hist, counters
        n = batch.n
        self.ws3 = engine.empty(16384 + 4 * (((n + 3) & ~3) + (1 << 22)), torch.uint8)
        sz = ctypes.c_size_t()
        engine.lib.avdb_vrs_digest_workspace_size(n, ctypes.byref(sz))
        self.ws4 = engine.empty(int(sz.value), torch.uint8)
        self.out: Dict[str, object] = {}

    def run(self, events: Optional[dict] = None) -> Dict[str, object]:
        """One step on the current stream: ``end, code, status, keep, digest, is_long``."""
        eng, b, msl = self.eng, self.b, self.max_seq_len
        main = torch.cuda.current_stream(eng.device)
        t = lambda name, fn: _timed(events, name, main, fn)  # noqa: E731
        end, code, status, _ = t("record_prep", lambda: eng.record_prep(
            b, want_lcp=False, hist=self.hist, counters=self.counters, max_seq_len=msl,
            digest_workspace=self.ws4, dedup_workspace=self.ws3))
        keep = t("pk_dedup", lambda: eng.pk_dedup(b, grouped=True, counters=self.counters, workspace=self.ws3))
        dig, is_long = t("vrs_digest", lambda: eng.vrs_digest(b, msl, workspace=self.ws4))
        self.out = dict(end=end, code=code, status=status, keep=keep, digest=dig, is_long=is_long)
        return self.out
