"""Device engine: one ``avdb_ctx`` per GPU plus torch-owned HBM buffers.

Everything here goes through ``libavdb_hip.so``; torch supplies device memory,
the current HIP stream and host<->device copies (plumbing, not compute).

Data layout in HBM (structure of arrays, one row per alt allele; see
``include/avdb.h``):

=============  =======  =====================================================
chrom          uint8    contig code (``chromosomes.CHROM_NAMES`` order)
pos            int32    1-based VCF POS (stored as u32 by the kernels)
end            int32    1-based inclusive end (optional, K1 only)
allele_off     int64    offset of REF in ``heap``; ALT follows REF
ref_len        int32
alt_len        int32
ext_id         int64    refSNP key (0 = none), see :func:`ext_id_key`
heap           uint8    concatenated raw REF+ALT bytes
=============  =======  =====================================================
"""

from __future__ import annotations

import ctypes
import os
import re
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from .chromosomes import CHROM_NAMES, N_CHROM, length_table


# ---------------------------------------------------------------------------
# record batch (SoA)
# ---------------------------------------------------------------------------
@dataclass
class RecordBatch:
    chrom: torch.Tensor
    pos: torch.Tensor
    allele_off: Optional[torch.Tensor] = None
    ref_len: Optional[torch.Tensor] = None
    alt_len: Optional[torch.Tensor] = None
    heap: Optional[torch.Tensor] = None
    ext_id: Optional[torch.Tensor] = None
    end: Optional[torch.Tensor] = None

    @property
    def n(self) -> int:
        return int(self.chrom.numel())

    @property
    def device(self):
        return self.chrom.device

    def to(self, device, non_blocking=False) -> "RecordBatch":
        kw = {}
        for f in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap", "ext_id", "end"):
            t = getattr(self, f)
            kw[f] = None if t is None else t.to(device, non_blocking=non_blocking)
        return RecordBatch(**kw)

    def has_alleles(self) -> bool:
        return self.heap is not None


_RS_RE = re.compile(r"^rs([1-9][0-9]{0,17})$")


class ExtIdInterner:
    """Maps external-id strings to the u64 ``ext_id`` keys the kernels compare.

    Canonical ``rs<N>`` ids map to ``N`` (N < 2^62); any other string gets
    ``2^63 | k`` for an interned index ``k``; ``None`` is 0.  Equal keys <=>
    equal strings, which is all the dedup contract needs."""

    def __init__(self):
        self._ids: Dict[str, int] = {}
        self._rev: List[str] = []

    def key(self, s: Optional[str]) -> int:
        if s is None:
            return 0
        m = _RS_RE.match(s)
        if m:
            return int(m.group(1))
        k = self._ids.get(s)
        if k is None:
            k = len(self._rev)
            self._ids[s] = k
            self._rev.append(s)
        return (1 << 63) | k

    def to_str(self, key: int) -> Optional[str]:
        if key == 0:
            return None
        if key >> 63:
            return self._rev[key & ((1 << 63) - 1)]
        return "rs%d" % key


def pack_records(chrom_codes: Sequence[int], pos: Sequence[int], refs: Sequence[bytes],
                 alts: Sequence[bytes], ext_ids: Optional[Sequence[int]] = None) -> RecordBatch:
    """Host-side SoA packing (numpy -> pinned CPU tensors)."""
    n = len(pos)
    rl = np.fromiter((len(r) for r in refs), dtype=np.int64, count=n)
    al = np.fromiter((len(a) for a in alts), dtype=np.int64, count=n)
    tot = rl + al
    off = np.zeros(n, dtype=np.int64)
    if n:
        np.cumsum(tot[:-1], out=off[1:])
    heap = b"".join(r + a for r, a in zip(refs, alts))
    heap_np = np.frombuffer(heap, dtype=np.uint8) if heap else np.zeros(1, dtype=np.uint8)
    ext = np.zeros(n, dtype=np.int64) if ext_ids is None else \
        np.asarray([int(x) if x < (1 << 63) else int(x) - (1 << 64) for x in ext_ids], dtype=np.int64)
    return RecordBatch(
        chrom=torch.from_numpy(np.asarray(chrom_codes, dtype=np.uint8)),
        pos=torch.from_numpy(np.asarray(pos, dtype=np.int64).astype(np.int32)),
        allele_off=torch.from_numpy(off),
        ref_len=torch.from_numpy(rl.astype(np.int32)),
        alt_len=torch.from_numpy(al.astype(np.int32)),
        heap=torch.from_numpy(heap_np.copy()),
        ext_id=torch.from_numpy(ext),
    )


def as_u32(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy().view(np.uint32)


# avdb_vcf_line (include/avdb.h), 80 bytes
VCF_LINE_DTYPE = np.dtype([("start", "<u8"), ("len", "<u4"), ("n_fields", "<u4"), ("field", "<u4", (8,)),
                           ("field_end8", "<u4"), ("pos", "<u4"), ("ext_id", "<u8"), ("n_alt", "<u4"),
                           ("n_rec", "<u4"), ("flags", "<u4"), ("chrom", "u1"), ("pad", "u1", (3,))])
assert VCF_LINE_DTYPE.itemsize == 80

VCF_COMMENT = 0x001
VCF_FEW_FIELDS = 0x002
VCF_BAD_POS = 0x004
VCF_EXT_HOST = 0x008
VCF_ID_RS = 0x010
VCF_INFO_RS = 0x020
VCF_ID_METASEQ = 0x040
VCF_CHROM_HOST = 0x080
VCF_EMPTY = 0x100
VCF_ID_HOST = 0x200
VCF_HOST_FLAGS = VCF_BAD_POS | VCF_EXT_HOST | VCF_CHROM_HOST | VCF_ID_HOST


def _stamp(*ts) -> tuple:
    """Identity + version of each tensor: what a keyed K2 hand-off is tied to.
    A weak reference (a freed tensor whose block the caching allocator hands to a
    new tensor at the same address does not match) and ``_version`` (an in-place
    edit of the batch between the producer and the consumer does not match)."""
    import weakref
    return tuple(None if t is None else (weakref.ref(t), t._version) for t in ts)


def _stamp_ok(stamp: tuple, *ts) -> bool:
    if stamp is None or len(stamp) != len(ts):
        return False
    for st, t in zip(stamp, ts):
        if st is None or t is None:
            if st is not None or t is not None:
                return False
        elif st[0]() is not t or t._version != st[1]:
            return False
    return True


@dataclass
class VcfBatch:
    """Output of ``Engine.vcf_tokenize``: device text, per-line table, records."""
    text: torch.Tensor
    n_lines: int
    lines: Optional[torch.Tensor]  # uint8[n_lines * 80] (VCF_LINE_DTYPE); None: vcf_tokenize(want_lines=False)
    rec_off: torch.Tensor        # int64[n_lines + 1]
    heap_off: torch.Tensor
    records: RecordBatch
    rec_line: torch.Tensor       # int32[n_rec]
    rec_alt: torch.Tensor

    def lines_host(self) -> np.ndarray:
        if self.lines is None:
            raise ValueError("this batch was tokenized without its line table (want_lines=False)")
        if self.n_lines == 0:
            return np.zeros(0, dtype=VCF_LINE_DTYPE)
        return self.lines.cpu().numpy()[: self.n_lines * 80].view(VCF_LINE_DTYPE)


class _Timer:
    """Optional HIP-event pairs on the engine's stream (bench stage timing)."""

    def __init__(self, events: Optional[dict], device):
        self.events, self.device, self.cur = events, device, None

    def start(self, name):
        if self.events is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.device))
            self.cur = (name, e)

    def stop(self):
        if self.events is not None and self.cur:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.device))
            self.events.setdefault(self.cur[0], []).append((self.cur[1], e))
            self.cur = None


@dataclass
class FormatResult:
    """Output of ``Engine.vcf_format`` (device tensors)."""
    copy: torch.Tensor           # uint8: COPY rows of every GPU-rendered line, in line order
    mapping: torch.Tensor        # uint8: .mapping lines
    copy_off: torch.Tensor       # int64[n_lines + 1]: start of each line's rows
    map_off: torch.Tensor        # int64[n_lines + 1]
    line_state: torch.Tensor     # uint8[n_lines]: LINE_GPU / LINE_HOST / LINE_SKIP
    counters: torch.Tensor


@dataclass
class KeyText:
    """Output of ``Engine.primary_keys`` (device tensors): key i is
    ``keys[key_off[i]:key_off[i+1]]`` when ``state[i] == KEY_OK``; path i is
    ``paths[path_off[i]:path_off[i+1]]`` (empty for an unmappable record).
    ``off32``: ``key_off`` / ``path_off`` are raw buffers in the narrow layout
    (AVDB_KEYS_OFF32: uint32 low words + a uint64 base per 4,096 records) —
    :meth:`key_offsets` / :meth:`path_offsets` give the int64 offsets either way."""
    ws: torch.Tensor
    key_off: torch.Tensor
    path_off: Optional[torch.Tensor]
    state: torch.Tensor
    keys: Optional[torch.Tensor]
    paths: Optional[torch.Tensor]
    off32: bool = False

    @staticmethod
    def _wide(t: torch.Tensor, n: int) -> torch.Tensor:
        lb = (4 * (n + 1) + 7) & ~7
        low = t[: 4 * (n + 1)].view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        base = t[lb: lb + 8 * ((n >> 12) + 1)].view(torch.int64).repeat_interleave(4096)[: n + 1]
        return base + ((low - (base & 0xFFFFFFFF)) & 0xFFFFFFFF)

    def key_offsets(self, n: int) -> torch.Tensor:
        """int64 key offsets [n + 1] (device)."""
        return self._wide(self.key_off, n) if self.off32 else self.key_off[: n + 1]

    def path_offsets(self, n: int) -> Optional[torch.Tensor]:
        if self.path_off is None:
            return None
        return self._wide(self.path_off, n) if self.off32 else self.path_off[: n + 1]

    def host(self, n: int):
        """(keys, paths) as Python lists of str (None where not rendered).
        Raises ``ValueError`` if a text did not fit its buffer (a reused
        ``KeyText`` too small for this batch: state KEY_OVERFLOW / PATH_OVERFLOW)."""
        ko = self.key_offsets(n).cpu().numpy()
        kb = self.keys[: int(ko[n])].cpu().numpy().tobytes()
        st = self.state[:n].cpu().numpy()
        if ((st == N.KEY_OVERFLOW) | ((st & N.PATH_OVERFLOW) != 0)).any():
            raise ValueError("primary_keys: key/path text exceeded the reused KeyText buffers")
        keys = [kb[ko[i]:ko[i + 1]].decode() if st[i] == N.KEY_OK else None for i in range(n)]
        paths = None
        if self.paths is not None:
            po = self.path_offsets(n).cpu().numpy()
            pb = self.paths[: int(po[n])].cpu().numpy().tobytes()
            paths = [pb[po[i]:po[i + 1]].decode() or None for i in range(n)]
        return keys, paths


class SmallPrep:
    """K8 (``avdb_small_prep``) over one host-mapped pinned arena: the
    per-record / per-line drop-in path as one launch + one stream sync, no
    copies (the kernel reads the records and writes the results over PCIe).
    Batches that do not fit the arena return ``None`` (callers then use the
    multi-kernel path).

    A call of at most ``host_max`` records (one ``find_bin_index`` miss, one
    ``parse_variant`` line) runs K8h instead, ``avdb_small_prep_host``: the
    same record arithmetic compiled into the library's host code, over the same
    arena.  A launch plus a stream sync costs ~25 us on MI355X, more than the
    reference's whole per-line call; the kernels take every batch.
    ``AVDB_PERCALL=gpu`` (or ``mode='gpu'``) sends every call to K8,
    ``AVDB_PERCALL=host`` every call that fits to K8h."""

    HOST_MAX = 32

    def __init__(self, engine: "Engine", max_records: int = 4096, heap_bytes: int = 1 << 20,
                 text_bytes: Tuple[int, int, int] = (1 << 19, 1 << 19, 1 << 21)):
        self.eng = engine
        self.mode = os.environ.get("AVDB_PERCALL", "auto")  # auto | host | gpu
        self.host_max = self.HOST_MAX
        self.last_path = None  # "host" | "gpu": which entry served the last call
        self.R = int(max_records)
        self.H = int(heap_bytes)
        self.T = tuple(int(t) for t in text_bytes)
        # arena: the per-call SoA region (inputs then outputs of one call, packed
        # per call size by _layout: <= 62 bytes per record), the allele heap and
        # the three text streams
        self.scratch = 64 * (self.R + 1)
        regions = [("soa", self.scratch), ("heap", self.H)] + [("text%d" % k, self.T[k]) for k in range(3)]
        total = 0
        self.addr = {}
        offs = {}
        for name, nbytes in regions:
            total = (total + 63) & ~63
            offs[name] = total
            total += nbytes
        self._ptr = self._alloc(total)
        self._buf = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(self._ptr))
        self._mv = memoryview(self._buf).cast("B")
        self._layouts = {}
        for name, off in offs.items():
            self.addr[name] = self._ptr + off
        self._heap0 = offs["heap"]
        self._text0 = [offs["text%d" % k] for k in range(3)]

    def _alloc(self, total: int) -> int:
        """The arena: pinned host memory mapped into the device (avdb_host_alloc);
        plain host memory for a host-only engine (K8h never reads it from a kernel)."""
        if self.eng.host_only:
            self._host_arena = np.zeros(total + 64, dtype=np.uint8)
            return (self._host_arena.ctypes.data + 63) & ~63
        p = ctypes.c_void_p()
        N.check("avdb_host_alloc", self.eng.lib.avdb_host_alloc(total, ctypes.byref(p)))
        return p.value

    def close(self):
        if getattr(self, "_ptr", None):
            if not self.eng.host_only:
                self.eng.lib.avdb_host_free(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _layout(self, n: int, kind: int):
        """Per-call layout for ``n`` records (cached): the arrays of one call
        packed back to back at the start of the arena, a ``SmallBatch`` holding
        their pointers, and one ``struct`` each for all inputs and all outputs.
        kind: 0 intervals (end_in), 1 alleles, 2 alleles + ext_id."""
        key = (n, kind)
        lay = self._layouts.get(key)
        if lay is not None:
            return lay
        fmt_in, fmt_out = ["<"], ["<"]
        at = [0]
        ptr = {}

        def put(fmt, name, code, cnt, size):
            pad = (-at[0]) % 8
            if pad:
                fmt.append("%dx" % pad)
                at[0] += pad
            ptr[name] = self._ptr + at[0]
            fmt.append("%d%s" % (cnt, code))
            at[0] += cnt * size
        put(fmt_in, "chrom", "B", n, 1)
        put(fmt_in, "pos", "I", n, 4)
        if kind == 0:
            put(fmt_in, "end_in", "I", n, 4)
        else:
            put(fmt_in, "allele_off", "Q", n, 8)
            put(fmt_in, "ref_len", "I", n, 4)
            put(fmt_in, "alt_len", "I", n, 4)
            if kind == 2:
                put(fmt_in, "ext_id", "Q", n, 8)
        in_bytes = at[0] = (at[0] + 15) & ~15
        put(fmt_out, "end_out", "I", n, 4)
        put(fmt_out, "code", "I", n, 4)
        put(fmt_out, "status", "B", n, 1)
        if kind:
            put(fmt_out, "key_state", "B", n, 1)
            put(fmt_out, "disp_state", "B", n, 1)
        put(fmt_out, "off_out", "I", 3 * (n + 1), 4)
        put(fmt_out, "overflow", "I", 2, 4)
        if at[0] > self.scratch:
            return None
        b = N.SmallBatch()
        for name in ("chrom", "pos", "end_in", "allele_off", "ref_len", "alt_len", "ext_id", "end_out", "code",
                     "status", "key_state", "disp_state", "off_out", "overflow"):
            if name in ptr:
                setattr(b, name, ptr[name])
        b.heap = self.addr["heap"]
        for k in range(3):
            b.text_out[k] = self.addr["text%d" % k]
            b.text_cap[k] = self.T[k]
        b.n = n
        lay = (b, struct.Struct("".join(fmt_in)), struct.Struct("".join(fmt_out)), in_bytes)
        self._layouts[key] = lay
        return lay

    def run(self, chrom, pos, ends=None, refs: Optional[Sequence[bytes]] = None,
            alts: Optional[Sequence[bytes]] = None, ext=None, want: int = 1, max_seq_len: int = 50):
        """Returns a dict of results (lists) or ``None`` when the batch does not
        fit.  Text streams: ``path`` / ``key`` / ``display`` lists of str (None
        where not rendered).  All inputs of a call go into the arena with one
        ``struct.pack_into`` and all outputs come back with one ``unpack_from``
        (plus the allele bytes and the texts): a call of a few records costs a
        few microseconds of Python around the library call."""
        n = len(pos)
        if n > self.R:
            return None
        kind = 0 if refs is None else (2 if ext is not None else 1)
        lay = self._layout(n, kind)
        if lay is None:
            return None
        b, s_in, s_out, in_bytes = lay
        mv = self._mv
        if kind:
            rl = [len(x) for x in refs]
            al = [len(x) for x in alts]
            heap = b"".join([r + x for r, x in zip(refs, alts)])
            hb = len(heap)
            if hb > self.H:
                return None
            offs = [0] * n
            t = 0
            for i in range(n):
                offs[i] = t
                t += rl[i] + al[i]
            h0 = self._heap0
            mv[h0:h0 + hb] = heap
            b.heap_bytes = max(hb, 1)
            if kind == 2:
                s_in.pack_into(mv, 0, *chrom, *pos, *offs, *rl, *al, *ext)
            else:
                s_in.pack_into(mv, 0, *chrom, *pos, *offs, *rl, *al)
        else:
            s_in.pack_into(mv, 0, *chrom, *pos, *ends)
        b.max_seq_len, b.want = int(max_seq_len), int(want)
        on_host = self.mode == "host" or (self.mode == "auto" and n <= self.host_max) or self.eng.host_only
        if on_host:
            N.check("avdb_small_prep_host", self.eng.lib.avdb_small_prep_host(self.eng.ctx, ctypes.byref(b)))
        else:
            N.check("avdb_small_prep", self.eng.lib.avdb_small_prep(self.eng.ctx, ctypes.byref(b),
                                                                    self.eng._stream()))
            torch.cuda.current_stream(self.eng.device).synchronize()
        self.last_path = "host" if on_host else "gpu"
        r = s_out.unpack_from(mv, in_bytes)
        if r[-2] & want:  # overflow
            return None
        out = {"end": list(r[:n]), "code": list(r[n:2 * n]), "status": list(r[2 * n:3 * n])}
        k0 = 3 * n
        if kind:
            out["key_state"] = list(r[k0:k0 + n])
            out["disp_state"] = list(r[k0 + n:k0 + 2 * n])
            k0 += 2 * n
        for k, name in enumerate(("path", "key", "display")):
            if not (want >> k) & 1:
                continue
            o = r[k0 + k * (n + 1): k0 + (k + 1) * (n + 1)]
            t0 = self._text0[k]
            raw = bytes(mv[t0:t0 + o[n]]).decode("ascii")
            out[name] = [raw[o[i]:o[i + 1]] if o[i + 1] > o[i] else None for i in range(n)]
        return out


class ChromMap:
    """``avdb_chrom_map`` of a ChromosomeMap's ``source_id -> chromosome`` dict
    (chromosome_map_parser.py:51-91).  For each source id the host decides once
    what the reference's per-line code makes of it — ``update_chromosome`` then
    ``get_variant`` (xstr, 'MT' -> 'M', 'chr' removed, vcf_parser.py:117-155) —
    and gives the kernels the contig code, or 0xFF (the line is rendered by the
    host) when the result is not a canonical contig label, or when the source id
    is text Python would coerce to a number (a CHROM field equal to it becomes an
    int before the lookup and never matches: KeyError)."""

    def __init__(self, engine: "Engine", mapping: Dict):
        from .chromosomes import CHROM_NAMES as names, bin_index_chrom_code
        from .parsers import to_numeric
        self.eng, self.mapping = engine, mapping
        keys, codes = [], []
        for k, v in mapping.items():
            if not isinstance(k, str):
                continue  # a CHROM field is a str (or a number): never this key
            try:
                kb = k.encode("ascii")
            except UnicodeEncodeError:
                continue  # K0 flags non-ASCII lines for the host anyway
            chrom = "" if v is None else str(v)
            if chrom == "MT":
                chrom = "M"
            chrom = chrom.replace("chr", "")
            c = bin_index_chrom_code(chrom)
            ok = c < len(names) and names[c] == chrom and isinstance(to_numeric(k), str)
            keys.append(kb)
            codes.append(c if ok else 0xFF)
        off = np.zeros(len(keys) + 1, dtype=np.uint64)
        if keys:
            off[1:] = np.cumsum([len(k) for k in keys])
        blob = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
        cd = np.asarray(codes or [0], dtype=np.uint8)
        h = ctypes.c_void_p()
        N.check("avdb_chrom_map_create", engine.lib.avdb_chrom_map_create(
            engine.ctx, blob.ctypes.data, off.ctypes.data, len(keys), cd.ctypes.data, ctypes.byref(h)))
        self.handle = h.value
        self.n_keys = len(keys)

    def close(self):
        if getattr(self, "handle", None):
            self.eng.lib.avdb_chrom_map_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LineHost:
    """K5h (``avdb_vcf_line_host``): one VCF line -> its COPY rows and .mapping
    line, rendered by the library's host code with the kernels' own per-line
    definitions (K0 parse_line, K2 infer_end/classify, K5 format_line).  The
    loader's per-line ``parse_variant`` uses it: no GPU launch per line."""

    def __init__(self, engine: "Engine", cap: int = 1 << 16):
        self.eng = engine
        self.res = N.LineResult()
        self.opts = N.FormatOpts()
        self.rendered = 0  # lines this entry rendered (the rest went to the caller)
        self._grow(cap)

    def _grow(self, cap: int):
        self.cap = int(cap)
        self._copy = ctypes.create_string_buffer(self.cap)
        self._map = ctypes.create_string_buffer(self.cap)
        self._ca, self._ma = ctypes.addressof(self._copy), ctypes.addressof(self._map)

    def run(self, line: bytes, alg_id: bytes, max_seq_len: int = 50, adsp: bool = False, vcf_opts=None):
        """``(state, copy_text, mapping_text, result)``; the texts are None unless
        state == LINE_GPU (rendered).  ``vcf_opts``: header width / chromosome map."""
        o = self.opts
        o.alg_id, o.max_seq_len, o.flags = alg_id, max_seq_len, N.FORMAT_ADSP if adsp else 0
        r = self.res
        vo = ctypes.byref(vcf_opts) if vcf_opts is not None else None
        rc = self.eng.lib.avdb_vcf_line_host(self.eng.ctx, line, len(line), ctypes.byref(o), vo, self._ca, self.cap,
                                             self._ma, self.cap, ctypes.byref(r))
        if rc == N.AVDB_ERANGE:
            self._grow(2 * max(r.copy_bytes, r.map_bytes))
            rc = self.eng.lib.avdb_vcf_line_host(self.eng.ctx, line, len(line), ctypes.byref(o), vo, self._ca,
                                                 self.cap, self._ma, self.cap, ctypes.byref(r))
        N.check("avdb_vcf_line_host", rc)
        if r.state != N.LINE_GPU:
            return r.state, None, None, r
        self.rendered += 1
        return (r.state, ctypes.string_at(self._ca, r.copy_bytes).decode("ascii"),
                ctypes.string_at(self._ma, r.map_bytes).decode("ascii"), r)


# ---------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------
class Engine:
    """A context on one GPU: chromosome-length table + kernel entry points."""

    def __init__(self, device=None, lengths: Optional[Sequence[int]] = None, assembly: str = "GRCh38",
                 sequence_digests: Optional[Sequence[str]] = None):
        if device is None and os.environ.get("AVDB_DEVICE") == "host":
            device = "host"
        # "host": a host-only engine — only the library's per-call host entries
        # (K5h, K8h, K1h: the kernels' record arithmetic compiled for the host side)
        # work; every kernel entry raises NativeUnavailable.  Opt-in only
        # (device="host" or AVDB_DEVICE=host), never a silent fallback.
        self.host_only = device == "host"
        if not self.host_only:
            N.require_gpu()
        self.lib = N.load_library()
        if self.host_only:
            self.device = torch.device("cpu")
        else:
            if device is None:
                device = torch.cuda.current_device()
            self.device = torch.device("cuda", int(device) if not isinstance(device, torch.device)
                                       else (device.index or 0))
        self.lengths = list(lengths) if lengths is not None else length_table(assembly)
        arr = (ctypes.c_uint32 * len(self.lengths))(*self.lengths)
        h = ctypes.c_void_p()
        N.check("avdb_ctx_create", self.lib.avdb_ctx_create(-1 if self.host_only else self.device.index, arr,
                                                            len(self.lengths), ctypes.byref(h)))
        self._ctx = h
        nb = ctypes.c_uint32()
        self.lib.avdb_l8_bin_count(self._ctx, ctypes.byref(nb))
        self.n_l8 = int(nb.value)
        # what the last keyed K2 left for its consumers, each entry tied (by _stamp)
        # to the exact tensors it was computed from and taken by the one call it
        # was meant for: "totals" (K7's group totals in a KeyText's workspace),
        # "codes" (K4's long-record codes in a digest workspace), "marks" (K3's
        # first phase in a dedup workspace + keep).  Every record_prep call drops
        # all of them first.
        self._pending: Dict[str, tuple] = {}
        self.last_vcf_path = ""  # vcf_tokenize(want_lines=False): "local" (count-free) or "counted"
        # test hook: every output / workspace tensor the engine allocates is filled
        # with this byte first (None: torch.empty), so a check sees only what the
        # kernels wrote, never what an earlier pass left in a recycled block
        self.poison: Optional[int] = None
        if sequence_digests is not None:
            self.set_sequence_digests(sequence_digests)

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if getattr(self, "_small", None) is not None:
            self._small.close()
            self._small = None
        if getattr(self, "_ctx", None):
            self.lib.avdb_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        if not self._ctx:
            raise N.NativeUnavailable("engine closed")
        return self._ctx

    def _stream(self):
        if self.host_only:
            raise N.NativeUnavailable("a host-only engine (AVDB_DEVICE=host) runs the per-call host entries only; "
                                      "this batch entry is a gfx950 kernel and needs a GPU")
        return N.stream_handle(self.device)

    def small(self) -> SmallPrep:
        """The engine's K8 arena (created on first use)."""
        sp = getattr(self, "_small", None)
        if sp is None:
            sp = self._small = SmallPrep(self)
        return sp

    def chrom_map(self, mapping: Dict, key=None) -> "ChromMap":
        """A ChromosomeMap's ``source_id -> chromosome`` dict as a library map
        (device table for K0, host table for K5h), cached per ``key``."""
        cache = self.__dict__.setdefault("_chrom_maps", {})
        k = key if key is not None else id(mapping)
        cm = cache.get(k)
        if cm is None or cm.mapping is not mapping:
            cm = cache[k] = ChromMap(self, mapping)
        return cm

    def vcf_opts(self, min_fields: int = 0, chrom_map: Optional["ChromMap"] = None) -> "N.VcfOpts":
        return N.VcfOpts(min_fields, chrom_map.handle if chrom_map is not None else None)

    def line_host(self) -> LineHost:
        """The engine's K5h per-line renderer (created on first use)."""
        lh = getattr(self, "_line_host", None)
        if lh is None:
            lh = self._line_host = LineHost(self)
        return lh

    def set_sequence_digests(self, digests: Sequence[str]):
        if len(digests) != len(self.lengths) or any(len(d) != N.DIGEST_CHARS for d in digests):
            raise ValueError("need one 32-character refget digest per chromosome")
        blob = "".join(digests).encode("ascii")
        N.check("avdb_ctx_set_sequence_digests",
                self.lib.avdb_ctx_set_sequence_digests(self.ctx, blob, len(digests)))

    # -- buffers -----------------------------------------------------------
    def empty(self, n, dtype):
        t = torch.empty(n, dtype=dtype, device=self.device)
        if self.poison is not None:
            t.view(torch.uint8).fill_(self.poison)
        return t

    def scratch(self, name: str, nbytes: int) -> torch.Tensor:
        """A workspace of at least ``nbytes`` bytes kept by the engine under ``name``
        and reused by later calls (grown when too small).  Every user runs on the
        engine's stream, so a later call's kernels are ordered after the earlier
        call's; with ``poison`` set it is refilled like a fresh buffer."""
        cache = self.__dict__.setdefault("_scratch", {})
        t = cache.get(name)
        if t is None or t.numel() < nbytes or t.device != self.device:
            cache[name] = None
            t = cache[name] = torch.empty(max(1, int(nbytes)), dtype=torch.uint8, device=self.device)
        if self.poison is not None:
            t.fill_(self.poison)
        return t

    def set_option(self, option: int, value: int):
        """``avdb_ctx_set_option`` (launch shape only: ``N.OPT_K4_GRID``)."""
        N.check("avdb_ctx_set_option", self.lib.avdb_ctx_set_option(self.ctx, int(option), int(value)))

    def new_histogram(self) -> torch.Tensor:
        return torch.zeros(self.n_l8, dtype=torch.int32, device=self.device)

    def new_counters(self) -> torch.Tensor:
        return torch.zeros(N.N_COUNTERS, dtype=torch.int64, device=self.device)

    def _dev(self, t: Optional[torch.Tensor]):
        if t is None:
            return None
        if t.device != self.device:
            t = t.to(self.device, non_blocking=True)
        return t.contiguous()

    # -- K1 ----------------------------------------------------------------
    def bin_assign(self, chrom: torch.Tensor, start: torch.Tensor, end: Optional[torch.Tensor] = None,
                   *, want_status: bool = True, hist: Optional[torch.Tensor] = None,
                   counters: Optional[torch.Tensor] = None,
                   out_code: Optional[torch.Tensor] = None,
                   out_status: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        chrom, start, end = self._dev(chrom), self._dev(start), self._dev(end)
        n = chrom.numel()
        if start.numel() != n or (end is not None and end.numel() != n):
            raise ValueError("chrom/start/end length mismatch")
        if chrom.dtype != torch.uint8 or start.element_size() != 4 or (end is not None and end.element_size() != 4):
            raise TypeError("chrom must be uint8, start/end 32-bit")
        code = out_code if out_code is not None else self.empty(n, torch.int32)
        status = None
        if want_status:
            status = out_status if out_status is not None else self.empty(n, torch.uint8)
        if hist is not None and hist.numel() != self.n_l8:
            raise ValueError("histogram must have n_l8 bins")
        N.check("avdb_bin_assign", self.lib.avdb_bin_assign(
            self.ctx, N.ptr(chrom), N.ptr(start), N.ptr(end), n, N.ptr(code), N.ptr(status),
            N.ptr(hist), N.ptr(counters), self._stream()))
        return code, status

    # -- K2 ----------------------------------------------------------------
    def record_prep(self, b: RecordBatch, *, want_lcp: bool = True, hist: Optional[torch.Tensor] = None,
                    counters: Optional[torch.Tensor] = None, keys: Optional["KeyText"] = None,
                    key_digest: bool = False, key_paths: bool = True, max_seq_len: int = 50,
                    digest_workspace: Optional[torch.Tensor] = None,
                    dedup_workspace: Optional[torch.Tensor] = None):
        """Returns ``(end, code, status, lcp)`` device tensors.  With ``keys`` (a
        one-pass ``KeyText`` from an earlier ``primary_keys`` on a same-sized
        batch) K2 also writes K7's group totals into its workspace
        (``avdb_record_prep_keyed``), so the next ``primary_keys(b, code,
        digest if key_digest, out=keys)`` skips its totals pass; with
        ``digest_workspace`` too (the K4 workspace the next ``vrs_digest(b,
        max_seq_len, workspace=...)`` gets) it classifies the long records for K4,
        and with ``dedup_workspace`` (the one the next ``pk_dedup(b, workspace=...)``
        gets) it runs K3's first phase, so that call only resolves the listed runs.
        Either workspace without ``keys`` runs the same K2 without K7's totals (a
        step with no key text, as C5's)."""
        b = b if b.device == self.device else b.to(self.device)
        n = b.n
        self._check_alleles(b)
        self._pending.clear()
        end = self.empty(n, torch.int32)
        code = self.empty(n, torch.int32)
        status = self.empty(n, torch.uint8)
        lcp = self.empty(n, torch.int32) if want_lcp else None
        args = (self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len),
                N.ptr(b.alt_len), N.ptr(b.heap), b.heap.numel(), n, N.ptr(end), N.ptr(code), N.ptr(status),
                N.ptr(lcp), N.ptr(hist), N.ptr(counters))
        if keys is None and digest_workspace is None and dedup_workspace is None:
            N.check("avdb_record_prep", self.lib.avdb_record_prep(*args, self._stream()))
            return end, code, status, lcp
        dws = digest_workspace
        if dws is not None:
            sz = ctypes.c_size_t()
            self.lib.avdb_vrs_digest_workspace_size(n, ctypes.byref(sz))
            if dws.numel() < sz.value:
                raise ValueError("record_prep: digest_workspace needs %d bytes" % sz.value)
        ddw = dedup_workspace
        keep = None
        if ddw is not None:
            keep = self.empty(max(4, n), torch.uint8)
        done = ctypes.c_int(0)
        N.check("avdb_record_prep_keyed", self.lib.avdb_record_prep_keyed(
            *args, N.ptr(b.ext_id), int(max_seq_len), 1 if key_digest else 0, 1 if key_paths else 0,
            N.ptr(keys.ws) if keys is not None else None, keys.ws.numel() if keys is not None else 0,
            N.ptr(dws), dws.numel() if dws is not None else 0,
            N.ptr(ddw), ddw.numel() if ddw is not None else 0, N.ptr(keep), ctypes.byref(done), self._stream()))
        # (tied to these exact tensors: another batch, a reallocated one or an
        # in-place edit recomputes)
        if done.value & N.KEYED_TOTALS:
            self._pending["totals"] = (_stamp(keys.ws, b.chrom, b.pos, b.ref_len, b.alt_len, b.ext_id,
                                              code if key_paths else None),
                                       keys, n, int(max_seq_len), bool(key_digest))
        if done.value & N.KEYED_LONG_CODES:
            self._pending["codes"] = (_stamp(dws, b.ref_len, b.alt_len), n, int(max_seq_len))
        if done.value & N.KEYED_DEDUP_MARKS:
            self._pending["marks"] = (_stamp(ddw, b.chrom, b.pos), n, keep)
        return end, code, status, lcp

    def keyed_prep(self, b: RecordBatch, kt: "KeyText", *, max_seq_len: int = 50, defer_digest: bool = True,
                   hist: Optional[torch.Tensor] = None, counters: Optional[torch.Tensor] = None,
                   digest_workspace: Optional[torch.Tensor] = None,
                   dedup_workspace: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None):
        """K2 + K7 in one pass (``avdb_keyed_prep``): ``(end, code, status, keep)``
        and ``kt`` filled with the keys and ltree paths (long keys' digests pending
        for :meth:`fill_digests` when ``defer_digest``).  With ``digest_workspace``
        (the one the next ``vrs_digest`` gets) it classifies the long records for K4;
        with ``dedup_workspace`` it runs K3's first phase (``keep`` = 1 and the listed
        runs; the next ``pk_dedup(b, workspace=...)`` resolves them), else ``keep`` is
        None.  ``workspace``: ``avdb_keyed_prep_workspace_size`` bytes (allocated
        when None)."""
        b = b if b.device == self.device else b.to(self.device)
        n = b.n
        self._check_alleles(b)
        self._pending.clear()
        if kt.key_off.numel() < n + 1 or kt.state.numel() < max(1, n) or kt.keys is None or kt.off32:
            raise ValueError("keyed_prep: the KeyText holds fewer records (or narrow offsets)")
        sz = ctypes.c_size_t()
        self.lib.avdb_keyed_prep_workspace_size(n, ctypes.byref(sz))
        ws = workspace if workspace is not None and workspace.numel() >= sz.value else \
            self.empty(int(sz.value), torch.uint8)
        end = self.empty(n, torch.int32)
        code = self.empty(n, torch.int32)
        status = self.empty(n, torch.uint8)
        dws, ddw = digest_workspace, dedup_workspace
        keep = self.empty(max(4, n), torch.uint8) if ddw is not None else None
        done = ctypes.c_int(0)
        N.check("avdb_keyed_prep", self.lib.avdb_keyed_prep(
            self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len), N.ptr(b.alt_len),
            N.ptr(b.heap), b.heap.numel(), N.ptr(b.ext_id), n, int(max_seq_len), N.ptr(end), N.ptr(code),
            N.ptr(status), N.ptr(hist), N.ptr(counters), N.ptr(ws), ws.numel(), N.ptr(dws),
            dws.numel() if dws is not None else 0, N.ptr(ddw), ddw.numel() if ddw is not None else 0, N.ptr(keep),
            N.ptr(kt.key_off), N.ptr(kt.path_off) if kt.paths is not None else None, N.ptr(kt.keys), kt.keys.numel(),
            N.ptr(kt.paths), kt.paths.numel() if kt.paths is not None else 0, N.ptr(kt.state),
            N.KEYS_DIGEST_DEFERRED if defer_digest else 0, ctypes.byref(done), self._stream()))
        self.last_keyed_ws = ws
        if done.value & N.KEYED_LONG_CODES:
            self._pending["codes"] = (_stamp(dws, b.ref_len, b.alt_len), n, int(max_seq_len))
        if done.value & N.KEYED_DEDUP_MARKS:
            self._pending["marks"] = (_stamp(ddw, b.chrom, b.pos), n, keep, N.DEDUP_ONEPASS)
        return end, code, status, keep

    def keyed_prep_lookback_errors(self, workspace: torch.Tensor) -> int:
        """Look-back polls that gave up in the last ``keyed_prep`` on ``workspace``
        (a host sync; 0 expected)."""
        v = ctypes.c_uint32()
        N.check("avdb_keyed_prep_lookback_errors",
                self.lib.avdb_keyed_prep_lookback_errors(self.ctx, N.ptr(workspace), ctypes.byref(v)))
        return int(v.value)

    # -- K3 ----------------------------------------------------------------
    def pk_dedup(self, b: RecordBatch, *, grouped: bool = True,
                 counters: Optional[torch.Tensor] = None,
                 workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
        b = b if b.device == self.device else b.to(self.device)
        n = b.n
        self._check_alleles(b)
        marks = self._pending.pop("marks", None)
        if (grouped and workspace is not None and marks is not None and marks[1] == n
                and _stamp_ok(marks[0], workspace, b.chrom, b.pos)):
            # the keyed K2 already wrote keep = 1 and listed the runs: resolve them
            keep = marks[2]
            flags = N.DEDUP_MARKED | (marks[3] if len(marks) > 3 else 0)
            N.check("avdb_pk_dedup_ex", self.lib.avdb_pk_dedup_ex(
                self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len),
                N.ptr(b.alt_len), N.ptr(b.heap), b.heap.numel(), N.ptr(b.ext_id), n, N.ptr(workspace),
                workspace.numel(), N.ptr(keep), N.ptr(counters), flags, self._stream()))
            return keep[:n]
        keep = self.empty(n, torch.uint8)
        ws = None
        ws_bytes = 0
        if grouped:  # optional list of same-position records (two-phase run scan)
            ws_bytes = 16384 + 4 * ((n + 3) & ~3)
            ws = workspace if workspace is not None and workspace.numel() >= ws_bytes else \
                self.empty(ws_bytes, torch.uint8)
        else:
            sz = ctypes.c_size_t()
            self.lib.avdb_pk_dedup_workspace_size(n, ctypes.byref(sz))
            ws_bytes = int(sz.value)
            ws = workspace if workspace is not None and workspace.numel() >= ws_bytes else \
                self.empty(ws_bytes, torch.uint8)
        N.check("avdb_pk_dedup", self.lib.avdb_pk_dedup(
            self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len),
            N.ptr(b.alt_len), N.ptr(b.heap), b.heap.numel(), N.ptr(b.ext_id), n, 1 if grouped else 0,
            N.ptr(ws), ws_bytes, N.ptr(keep), N.ptr(counters), self._stream()))
        return keep

    # -- K4 ----------------------------------------------------------------
    def vrs_digest(self, b: RecordBatch, max_seq_len: int = 50,
                   workspace: Optional[torch.Tensor] = None,
                   keys: Optional["KeyText"] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Returns ``(digests uint8[n,32], is_long uint8[n])``.  Only the rows
        with ``is_long`` set are written (the rest are unspecified: zero-filling
        32 bytes per record would cost more HBM traffic than the digests).
        ``keys``: the ``KeyText`` of a deferred ``primary_keys`` / ``keyed_prep``
        on this batch — the digests also go into its pending keys
        (``avdb_vrs_digest_keys``: no :meth:`fill_digests` pass)."""
        b = b if b.device == self.device else b.to(self.device)
        n = b.n
        self._check_alleles(b)
        dig = self.empty(max(1, n) * N.DIGEST_CHARS, torch.uint8).view(-1, N.DIGEST_CHARS)[:n]
        is_long = self.empty(n, torch.uint8)
        sz = ctypes.c_size_t()
        self.lib.avdb_vrs_digest_workspace_size(n, ctypes.byref(sz))
        ws = workspace if workspace is not None and workspace.numel() >= sz.value else \
            self.empty(int(sz.value), torch.uint8)
        # the keyed K2 classified this batch's records into this workspace
        codes = self._pending.pop("codes", None)
        ready = (codes is not None and codes[1:] == (n, int(max_seq_len))
                 and _stamp_ok(codes[0], ws, b.ref_len, b.alt_len))
        args = (self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len),
                N.ptr(b.alt_len), N.ptr(b.heap), b.heap.numel(), n, int(max_seq_len), N.ptr(ws), int(sz.value),
                N.ptr(dig), N.ptr(is_long), N.DIGEST_CODES_READY if ready else 0)
        if keys is None:
            N.check("avdb_vrs_digest_ex", self.lib.avdb_vrs_digest_ex(*args, self._stream()))
        else:
            if keys.off32:
                raise ValueError("vrs_digest(keys=...): narrow key offsets are not accepted")
            N.check("avdb_vrs_digest_keys", self.lib.avdb_vrs_digest_keys(
                *args, N.ptr(keys.key_off), N.ptr(keys.keys), N.ptr(keys.state), self._stream()))
        return dig, is_long

    def sha512t24u(self, blobs: Sequence[bytes]) -> List[str]:
        n = len(blobs)
        if n == 0:
            return []
        lens = np.fromiter((len(x) for x in blobs), dtype=np.int64, count=n)
        off = np.zeros(n, dtype=np.int64)
        np.cumsum(lens[:-1], out=off[1:])
        data = b"".join(blobs) or b"\0"
        d_data = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(self.device)
        d_off = torch.from_numpy(off).to(self.device)
        d_len = torch.from_numpy(lens.astype(np.int32)).to(self.device)
        out = self.empty(n * N.DIGEST_CHARS, torch.uint8)
        N.check("avdb_sha512t24u", self.lib.avdb_sha512t24u(
            self.ctx, N.ptr(d_data), N.ptr(d_off), N.ptr(d_len), n, N.ptr(out), self._stream()))
        raw = out.cpu().numpy().tobytes()
        return [raw[i * 32:(i + 1) * 32].decode("ascii") for i in range(n)]

    # -- K0: VCF text -> records ---------------------------------------------
    def vcf_tokenize(self, text, vcf_opts: Optional["N.VcfOpts"] = None, want_lines: bool = True,
                     count_free: bool = True) -> "VcfBatch":
        """Parse VCF data lines (bytes or a uint8 tensor) on the GPU into the
        record SoA (one row per ALT != '.') plus the per-line table.
        ``vcf_opts`` (:meth:`vcf_opts`): header width and chromosome map.
        ``want_lines=False``: no public line table (``VcfBatch.lines`` is None) — for
        callers that need only the records: the count-free path (avdb_vcf_parse_local:
        each parse window writes its lines to slots of its own, one scan of the window
        totals, avdb_vcf_emit_local), or, when a window holds more lines, records or allele
        bytes than its slots, count -> parse -> emit from 32-byte records in the parse
        workspace (also taken with ``count_free=False``)."""
        if not want_lines and count_free:
            vb, text = self._vcf_tokenize_local(text, vcf_opts)
            if vb is not None:
                self.last_vcf_path = "local"
                return vb
            # (a window overflowed its line slots: the counted path, on the text the
            # count-free attempt already put on the device)
        self.last_vcf_path = "counted"
        if isinstance(text, (bytes, bytearray, memoryview)):
            host = bytes(text)
            t = torch.frombuffer(bytearray(host) if host else bytearray(b"\n"), dtype=torch.uint8)
            if not host:
                t = t[:0]
            text_t = t.to(self.device)
            last_nl = host.endswith(b"\n") if host else True
        else:
            text_t = self._dev(text)
            last_nl = None  # (read with the newline count: one host sync, not two)
        nb = int(text_t.numel())
        tp = N.ptr(text_t) if nb else None
        s = self._stream()
        csz = ctypes.c_size_t()
        self.lib.avdb_vcf_count_workspace_size(nb, ctypes.byref(csz))  # (with the parse windows' counts)
        ws0 = self.empty(int(csz.value), torch.uint8)
        nl = torch.zeros(2, dtype=torch.int64, device=self.device)  # newlines, last byte
        N.check("avdb_vcf_count_lines", self.lib.avdb_vcf_count_lines(
            self.ctx, tp, nb, N.ptr(ws0), ws0.numel(), N.ptr(nl), s))
        if last_nl is None and nb:
            nl[1:2].copy_(text_t[-1:])
        got = nl.cpu()
        n_nl = int(got[0])
        if last_nl is None:
            last_nl = nb == 0 or int(got[1]) == 10
        n_lines = n_nl + (0 if (last_nl or nb == 0) else 1)
        sz = ctypes.c_size_t()
        self.lib.avdb_vcf_workspace_size(nb, n_lines, ctypes.byref(sz))
        ws = self.empty(int(sz.value), torch.uint8)
        lines = self.empty(max(1, n_lines) * VCF_LINE_DTYPE.itemsize, torch.uint8) if want_lines else None
        rec_off = self.empty(n_lines + 1, torch.int64)
        heap_off = self.empty(n_lines + 1, torch.int64)
        N.check("avdb_vcf_parse_lines2", self.lib.avdb_vcf_parse_lines2(
            self.ctx, tp, nb, n_lines, N.ptr(ws0), ws0.numel(), N.ptr(ws), ws.numel(), N.ptr(lines), N.ptr(rec_off),
            N.ptr(heap_off), ctypes.byref(vcf_opts) if vcf_opts is not None else None, s))
        if n_lines:
            tot = torch.stack([rec_off[n_lines], heap_off[n_lines]]).cpu().tolist()
        else:
            tot = [0, 0]
        n_rec, n_heap = int(tot[0]), int(tot[1])
        b = RecordBatch(chrom=self.empty(n_rec, torch.uint8), pos=self.empty(n_rec, torch.int32),
                        allele_off=self.empty(n_rec, torch.int64),
                        ref_len=self.empty(n_rec, torch.int32), alt_len=self.empty(n_rec, torch.int32),
                        heap=self.empty(max(1, n_heap), torch.uint8),
                        ext_id=self.empty(n_rec, torch.int64))
        rec_line = self.empty(n_rec, torch.int32)
        rec_alt = self.empty(n_rec, torch.int32)
        outs = (N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len), N.ptr(b.alt_len),
                N.ptr(b.ext_id), N.ptr(b.heap), N.ptr(rec_line), N.ptr(rec_alt), s)
        if n_rec and want_lines:
            N.check("avdb_vcf_emit", self.lib.avdb_vcf_emit(
                self.ctx, tp, nb, n_lines, N.ptr(lines), N.ptr(rec_off), N.ptr(heap_off), *outs))
        elif n_rec:
            N.check("avdb_vcf_emit_ws", self.lib.avdb_vcf_emit_ws(
                self.ctx, tp, nb, n_lines, N.ptr(ws), ws.numel(), N.ptr(rec_off), N.ptr(heap_off), *outs))
        return VcfBatch(text=text_t, n_lines=n_lines, lines=lines, rec_off=rec_off, heap_off=heap_off,
                        records=b, rec_line=rec_line, rec_alt=rec_alt)

    def _vcf_tokenize_local(self, text, vcf_opts):
        """vcf_tokenize(want_lines=False) without the count pass: (batch, device
        text), the batch None when a parse window overflowed its line slots (the
        caller then takes the counted path on the same device text).  The slot
        workspace (about 2.7x the text: line, record and heap slots, avdb.h) is the
        engine's, reused across calls."""
        if isinstance(text, (bytes, bytearray, memoryview)):
            host = bytes(text)
            t = torch.frombuffer(bytearray(host) if host else bytearray(b"\n"), dtype=torch.uint8)
            text_t = (t if host else t[:0]).to(self.device)
        else:
            text_t = self._dev(text)
        nb = int(text_t.numel())
        tp = N.ptr(text_t) if nb else None
        s = self._stream()
        sz = ctypes.c_size_t()
        self.lib.avdb_vcf_local_workspace_size(nb, ctypes.byref(sz))
        ws = self.scratch("vcf_local", int(sz.value))
        tot = torch.zeros(4, dtype=torch.int64, device=self.device)
        N.check("avdb_vcf_parse_local", self.lib.avdb_vcf_parse_local(
            self.ctx, tp, nb, N.ptr(ws), ws.numel(), ctypes.byref(vcf_opts) if vcf_opts is not None else None,
            N.ptr(tot), s))
        n_lines, n_rec, n_heap, overflow = (int(v) for v in tot.cpu().tolist())
        if overflow:
            return None, text_t
        b = RecordBatch(chrom=self.empty(n_rec, torch.uint8), pos=self.empty(n_rec, torch.int32),
                        allele_off=self.empty(n_rec, torch.int64),
                        ref_len=self.empty(n_rec, torch.int32), alt_len=self.empty(n_rec, torch.int32),
                        heap=self.empty(max(1, n_heap), torch.uint8),
                        ext_id=self.empty(n_rec, torch.int64))
        rec_line = self.empty(n_rec, torch.int32)
        rec_alt = self.empty(n_rec, torch.int32)
        rec_off = self.empty(n_lines + 1, torch.int64)
        heap_off = self.empty(n_lines + 1, torch.int64)
        if n_rec == 0:  # (no line has a record: every offset is 0)
            rec_off.zero_()
            heap_off.zero_()
        else:
            N.check("avdb_vcf_emit_local", self.lib.avdb_vcf_emit_local(
                self.ctx, tp, nb, N.ptr(ws), ws.numel(), N.ptr(rec_off), N.ptr(heap_off), N.ptr(b.chrom),
                N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len), N.ptr(b.alt_len), N.ptr(b.ext_id),
                N.ptr(b.heap), N.ptr(rec_line), N.ptr(rec_alt), s))
        return VcfBatch(text=text_t, n_lines=n_lines, lines=None, rec_off=rec_off, heap_off=heap_off,
                        records=b, rec_line=rec_line, rec_alt=rec_alt), text_t

    # -- K9: this rank's lines of a VCF text -----------------------------------
    def vcf_select(self, vb: "VcfBatch", assignment, rank: int, cut: int = 64_000_000) -> torch.Tensor:
        """The lines of ``vb`` that piece plan ``assignment`` gives to ``rank``
        (each + '\\n', file order) as a device text tensor."""
        from .shard import piece_table
        base, count, prank = piece_table(assignment, self.lengths, cut)
        n = vb.n_lines
        sz = ctypes.c_size_t()
        self.lib.avdb_shard_workspace_size(n, ctypes.byref(sz))
        ws = self.empty(max(1, int(sz.value)), torch.uint8)
        sel = self.empty(n + 1, torch.int64)
        s = self._stream()
        N.check("avdb_vcf_select_lines", self.lib.avdb_vcf_select_lines(
            self.ctx, n, N.ptr(vb.lines), base.ctypes.data, count.ctypes.data, prank.ctypes.data, len(prank),
            int(cut), int(rank), N.ptr(ws), ws.numel(), N.ptr(sel), s))
        total = int(sel[n].item())
        out = self.empty(max(1, total), torch.uint8)
        if total:
            N.check("avdb_vcf_select_copy", self.lib.avdb_vcf_select_copy(
                self.ctx, N.ptr(vb.text), vb.text.numel(), n, N.ptr(vb.lines), N.ptr(sel), N.ptr(out), s))
        return out[:total]

    # -- K5: COPY rows / .mapping lines / display attributes --------------------
    def vcf_format(self, vb: "VcfBatch", end: torch.Tensor, code: torch.Tensor, status: torch.Tensor,
                   digest: Optional[torch.Tensor] = None, keep: Optional[torch.Tensor] = None,
                   alg_id="", max_seq_len: int = 50,
                   counters: Optional[torch.Tensor] = None, events: Optional[dict] = None,
                   existing: Optional[tuple] = None, adsp: bool = False,
                   adsp_dup: Optional[torch.Tensor] = None) -> "FormatResult":
        """The load driver's COPY buffer and .mapping text for ``vb``'s lines
        (K5b: size pass, scans, one host sync for the totals, write pass)."""
        n = vb.n_lines
        s = self._stream()
        tp = N.ptr(vb.text) if vb.text.numel() else None
        opts = N.FormatOpts(str(alg_id).encode(), int(max_seq_len), N.FORMAT_ADSP if adsp else 0)
        if adsp_dup is not None:  # ADSP: records whose primary key is already loaded
            opts.adsp_dup = N.ptr(adsp_dup)
        if existing is not None:  # (match, kind, frag, frag_off) device tensors from keyset_probe
            m, k, fr, fo = existing
            opts.match, opts.match_kind, opts.frag, opts.frag_off = N.ptr(m), N.ptr(k), N.ptr(fr), N.ptr(fo)
        if len(opts.alg_id) >= N.MAX_ALG_ID:
            raise ValueError("algorithm id too long")
        sz = ctypes.c_size_t()
        self.lib.avdb_format_workspace_size(n, ctypes.byref(sz))
        ws = self.empty(int(sz.value), torch.uint8)
        copy_off = self.empty(n + 1, torch.int64)
        map_off = self.empty(n + 1, torch.int64)
        state = self.empty(max(1, n), torch.uint8)
        if end.numel() == 0:  # no records in this batch: the kernels never read them
            end = code = self.empty(1, torch.int32)
            status = self.empty(1, torch.uint8)
        dg = None if digest is None else N.ptr(digest)
        kp = None if keep is None else N.ptr(keep)
        args = (self.ctx, tp, vb.text.numel(), n, N.ptr(vb.lines), N.ptr(vb.rec_off), N.ptr(end), N.ptr(code),
                N.ptr(status), dg, kp, ctypes.byref(opts))
        ev = _Timer(events, self.device)
        ev.start("format_size")
        N.check("avdb_vcf_format_size", self.lib.avdb_vcf_format_size(
            *args, N.ptr(ws), ws.numel(), N.ptr(copy_off), N.ptr(map_off), N.ptr(state), s))
        ev.stop()
        tot = torch.stack([copy_off[n], map_off[n]]).cpu().tolist()
        copy = self.empty(max(8, int(tot[0])), torch.uint8)
        mapping = self.empty(max(8, int(tot[1])), torch.uint8)
        ctr = counters if counters is not None else self.new_counters()
        ev.start("format_write")
        N.check("avdb_vcf_format_write", self.lib.avdb_vcf_format_write(
            *args, N.ptr(copy_off), N.ptr(map_off), N.ptr(state), N.ptr(copy), N.ptr(mapping), N.ptr(ctr), s))
        ev.stop()
        return FormatResult(copy=copy[: int(tot[0])], mapping=mapping[: int(tot[1])], copy_off=copy_off,
                            map_off=map_off, line_state=state[:n], counters=ctr)

    def display_attributes(self, b: RecordBatch, end: torch.Tensor):
        """K5a: json.dumps(get_display_attributes()) per record.  Returns
        ``(text uint8, off int64[n+1], state uint8[n])`` device tensors."""
        b = b if b.device == self.device else b.to(self.device)
        self._check_alleles(b)
        n = b.n
        s = self._stream()
        sz = ctypes.c_size_t()
        self.lib.avdb_format_workspace_size(n, ctypes.byref(sz))
        ws = self.empty(int(sz.value), torch.uint8)
        off = self.empty(n + 1, torch.int64)
        state = self.empty(max(1, n), torch.uint8)
        end = self._dev(end)
        args = (self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(end), N.ptr(b.allele_off), N.ptr(b.ref_len),
                N.ptr(b.alt_len), N.ptr(b.heap), b.heap.numel(), n, N.ptr(ws), ws.numel(), N.ptr(off))
        N.check("avdb_display_attributes", self.lib.avdb_display_attributes(*args, None, N.ptr(state), s))
        total = int(off[n].item())
        out = self.empty(max(8, total), torch.uint8)
        if n:
            N.check("avdb_display_attributes", self.lib.avdb_display_attributes(*args, N.ptr(out), N.ptr(state), s))
        return out[:total], off, state[:n]

    # -- K7: primary keys + bin paths as text ------------------------------------
    def primary_keys(self, b: RecordBatch, code: Optional[torch.Tensor] = None,
                     digest: Optional[torch.Tensor] = None, max_seq_len: int = 50, *,
                     out: Optional["KeyText"] = None, onepass: bool = True,
                     defer_digest: bool = False) -> "KeyText":
        """``generate_primary_key`` (and, with ``code``, the ltree bin path) for
        every record of ``b`` as text on the device.  Without ``out`` the size
        pass is followed by one host read of the totals; passing a ``KeyText``
        from an earlier call on a same-shaped batch reuses its buffers (no host
        sync: a text that would end past a buffer is not written and its record's
        state says so — ``KEY_OVERFLOW`` for the key, ``PATH_OVERFLOW`` ORed in
        for the path; ``KeyText.host`` raises on either).  ``defer_digest`` (no
        ``digest``): long records' keys are laid out with their 32 digest
        characters left for :meth:`fill_digests` (state ``KEY_DIGEST_PENDING``),
        so this launch need not wait for K4."""
        b = b if b.device == self.device else b.to(self.device)
        self._check_alleles(b)
        n = b.n
        s = self._stream()
        code = self._dev(code)
        digest = self._dev(digest)
        if defer_digest and (digest is not None or not onepass):
            raise ValueError("primary_keys: defer_digest takes no digest (one-pass form)")
        if onepass:
            return self._primary_keys_onepass(b, code, digest, max_seq_len, out, defer_digest)
        if out is None:
            sz = ctypes.c_size_t()
            self.lib.avdb_format_workspace_size(n, ctypes.byref(sz))
            out = KeyText(ws=self.empty(int(sz.value), torch.uint8), key_off=self.empty(n + 1, torch.int64),
                          path_off=self.empty(n + 1, torch.int64) if code is not None else None,
                          state=self.empty(max(1, n), torch.uint8), keys=None, paths=None)
        if out.off32:
            raise ValueError("primary_keys: narrow offsets need the one-pass form")
        if out.key_off.numel() < n + 1 or out.state.numel() < max(1, n) or \
                (code is not None and (out.path_off is None or out.path_off.numel() < n + 1)):
            raise ValueError("primary_keys: the reused KeyText holds fewer records (or no paths)")
        args = (self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len), N.ptr(b.alt_len),
                N.ptr(b.heap), b.heap.numel(), N.ptr(b.ext_id), N.ptr(code), N.ptr(digest), n, int(max_seq_len),
                N.ptr(out.ws), out.ws.numel(), N.ptr(out.key_off), N.ptr(out.path_off))
        N.check("avdb_primary_keys", self.lib.avdb_primary_keys(*args, None, 0, None, 0, None, s))
        if out.keys is None:
            tot = torch.stack([out.key_off[n], out.path_off[n] if code is not None else out.key_off[n]]).cpu().tolist()
            out.keys = self.empty(max(8, int(tot[0])), torch.uint8)
            out.paths = self.empty(max(8, int(tot[1])), torch.uint8) if code is not None else None
        if n:
            N.check("avdb_primary_keys", self.lib.avdb_primary_keys(
                *args, N.ptr(out.keys), out.keys.numel(), N.ptr(out.paths),
                out.paths.numel() if out.paths is not None else 0, N.ptr(out.state), s))
        return out

    def new_key_text(self, n: int, heap_bytes: int, paths: bool = True, off32: bool = False) -> "KeyText":
        """Buffers for one-pass K7 output over ``n`` records with ``heap_bytes`` of
        alleles (texts sized by ``avdb_primary_keys_bound``): what a keyed K2 writes
        its group totals into before the first ``primary_keys(..., out=...)``.
        ``off32``: the offsets in the narrow layout (AVDB_KEYS_OFF32, for exactly
        ``n`` records)."""
        sz = ctypes.c_size_t()
        self.lib.avdb_primary_keys_onepass_workspace_size(n, ctypes.byref(sz))
        kc, pc = ctypes.c_size_t(), ctypes.c_size_t()
        self.lib.avdb_primary_keys_bound(n, heap_bytes, ctypes.byref(kc), ctypes.byref(pc))
        if off32:
            ob = ctypes.c_size_t()
            self.lib.avdb_keys_off32_bytes(n, ctypes.byref(ob))
            mk = lambda: self.empty(int(ob.value), torch.uint8)  # noqa: E731
        else:
            mk = lambda: self.empty(n + 1, torch.int64)  # noqa: E731
        return KeyText(ws=self.empty(int(sz.value), torch.uint8), key_off=mk(), path_off=mk() if paths else None,
                       state=self.empty(max(16, n), torch.uint8), keys=self.empty(int(kc.value), torch.uint8),
                       paths=self.empty(int(pc.value), torch.uint8) if paths else None, off32=off32)

    def fill_digests(self, b: RecordBatch, digest: torch.Tensor, kt: "KeyText"):
        """``avdb_primary_keys_fill_digests``: the digest characters of every key a
        ``primary_keys(..., defer_digest=True)`` left pending (``digest`` = this
        batch's ``vrs_digest`` output)."""
        b = b if b.device == self.device else b.to(self.device)
        if kt.off32:
            raise ValueError("fill_digests: narrow key offsets are not accepted")
        N.check("avdb_primary_keys_fill_digests", self.lib.avdb_primary_keys_fill_digests(
            self.ctx, N.ptr(b.chrom), N.ptr(b.pos), b.n, N.ptr(digest), N.ptr(kt.key_off), N.ptr(kt.keys),
            N.ptr(kt.state), self._stream()))
        return kt

    def _primary_keys_onepass(self, b: RecordBatch, code, digest, max_seq_len: int, out,
                              defer: bool = False) -> "KeyText":
        """K7 without a host round trip (``avdb_primary_keys_onepass``): per-group
        size totals, two small scans, then the write pass that recomputes each
        record's sizes, writes its offsets and the text; the text buffers are sized
        by ``avdb_primary_keys_bound``, so no host sync is needed even the first time."""
        n = b.n
        sz = ctypes.c_size_t()
        self.lib.avdb_primary_keys_onepass_workspace_size(n, ctypes.byref(sz))
        if out is None:
            out = self.new_key_text(n, b.heap.numel(), paths=code is not None)
        if out.key_off.numel() < n + 1 or out.state.numel() < max(1, n) or \
                (code is not None and (out.path_off is None or out.path_off.numel() < n + 1 or out.paths is None)):
            raise ValueError("primary_keys: the reused KeyText holds fewer records (or no paths)")
        if out.off32:
            ob = ctypes.c_size_t()
            self.lib.avdb_keys_off32_bytes(n, ctypes.byref(ob))
            if out.key_off.numel() < ob.value or (code is not None and out.path_off.numel() < ob.value):
                raise ValueError("primary_keys: the narrow offset buffers were made for fewer records")
        if out.ws.numel() < sz.value:
            out.ws = self.empty(int(sz.value), torch.uint8)
        # the keyed K2 wrote this batch's group totals into this KeyText's workspace
        # (sizes from these length / id arrays and, for the paths, these bin codes)
        tot = self._pending.pop("totals", None)
        ready = (tot is not None and tot[1] is out and tot[2:] == (n, int(max_seq_len), digest is not None or defer)
                 and _stamp_ok(tot[0], out.ws, b.chrom, b.pos, b.ref_len, b.alt_len, b.ext_id, code))
        flags = (N.KEYS_TOTALS_READY if ready else 0) | (N.KEYS_DIGEST_DEFERRED if defer else 0) | \
            (N.KEYS_OFF32 if out.off32 else 0)
        N.check("avdb_primary_keys_onepass_ex", self.lib.avdb_primary_keys_onepass_ex(
            self.ctx, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len), N.ptr(b.alt_len),
            N.ptr(b.heap), b.heap.numel(), N.ptr(b.ext_id), N.ptr(code), N.ptr(digest), n, int(max_seq_len),
            N.ptr(out.ws), out.ws.numel(), N.ptr(out.key_off), N.ptr(out.path_off), N.ptr(out.keys), out.keys.numel(),
            N.ptr(out.paths), out.paths.numel() if out.paths is not None else 0, N.ptr(out.state),
            flags, self._stream()))
        return out

    # -- K6: existing-variant key set ----------------------------------------
    def keyset_build(self, keys: torch.Tensor, key_off: torch.Tensor) -> torch.Tensor:
        """Hash table over the key strings (``keys`` bytes, ``key_off`` int64[n+1])."""
        keys, key_off = self._dev(keys), self._dev(key_off)
        n = key_off.numel() - 1
        sz = ctypes.c_size_t()
        self.lib.avdb_keyset_workspace_size(n, ctypes.byref(sz))
        table = self.empty(int(sz.value), torch.uint8)
        N.check("avdb_keyset_build", self.lib.avdb_keyset_build(
            self.ctx, N.ptr(keys) if keys.numel() else None, N.ptr(key_off), n, N.ptr(table), table.numel(),
            self._stream()))
        return table

    def keyset_probe(self, table: torch.Tensor, keys: torch.Tensor, key_off: torch.Tensor, b: RecordBatch,
                     check_alt: bool = True, counters: Optional[torch.Tensor] = None):
        """``(match int32[n], kind uint8[n])``: first equal key of each record's
        metaseq id (then of the switched alleles with ``check_alt``)."""
        b = b if b.device == self.device else b.to(self.device)
        self._check_alleles(b)
        n = b.n
        match = self.empty(max(1, n), torch.int32)
        kind = self.empty(max(1, n), torch.uint8)
        N.check("avdb_keyset_probe", self.lib.avdb_keyset_probe(
            self.ctx, N.ptr(table), table.numel(), N.ptr(keys) if keys.numel() else None, N.ptr(key_off),
            key_off.numel() - 1, N.ptr(b.chrom), N.ptr(b.pos), N.ptr(b.allele_off), N.ptr(b.ref_len),
            N.ptr(b.alt_len), N.ptr(b.heap), b.heap.numel(), n, 1 if check_alt else 0, N.ptr(match), N.ptr(kind),
            N.ptr(counters), self._stream()))
        return match[:n], kind[:n]

    def keyset_probe_text(self, table: torch.Tensor, keys: torch.Tensor, key_off: torch.Tensor,
                          q: torch.Tensor, q_off: torch.Tensor, n: int, skip: Optional[torch.Tensor] = None,
                          counters: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``match int32[n]``: first key equal to ``q[q_off[i]:q_off[i+1]]``, or -1."""
        match = self.empty(max(1, n), torch.int32)
        N.check("avdb_keyset_probe_text", self.lib.avdb_keyset_probe_text(
            self.ctx, N.ptr(table), table.numel(), N.ptr(keys) if keys.numel() else None, N.ptr(key_off),
            key_off.numel() - 1, N.ptr(q) if q.numel() else None, N.ptr(q_off), N.ptr(skip), n, N.ptr(match),
            N.ptr(counters), self._stream()))
        return match[:n]

    # -- formatting (host) ---------------------------------------------------
    def format_path(self, chrom_code: int, code: int) -> Optional[str]:
        buf = ctypes.create_string_buffer(N.MAX_PATH)
        rc = self.lib.avdb_format_bin_path(self.ctx, chrom_code, code & 0xFFFFFFFF, buf, N.MAX_PATH)
        if rc < 0:
            return None
        return buf.raw[:rc].decode("ascii")

    def format_paths(self, chrom_codes: np.ndarray, codes: np.ndarray) -> List[Optional[str]]:
        """Host batch formatting of kernel outputs into ltree strings (None for
        unmappable rows)."""
        chrom_codes = np.ascontiguousarray(chrom_codes, dtype=np.uint8)
        codes = np.ascontiguousarray(codes).view(np.uint32)
        n = len(codes)
        cap = max(1, n * 88)
        out = np.empty(cap, dtype=np.uint8)
        offs = np.empty(n + 1, dtype=np.uint64)
        N.check("avdb_format_bin_paths", self.lib.avdb_format_bin_paths(
            self.ctx, chrom_codes.ctypes.data, codes.ctypes.data, n, out.ctypes.data, cap,
            offs.ctypes.data))
        raw = out[: int(offs[n])].tobytes().decode("ascii")
        res: List[Optional[str]] = []
        for i in range(n):
            a, b = int(offs[i]), int(offs[i + 1])
            res.append(raw[a:b] if b > a else None)
        return res

    @staticmethod
    def _check_alleles(b: RecordBatch):
        if not b.has_alleles():
            raise ValueError("batch has no allele heap")
        if b.allele_off.dtype != torch.int64 or b.ref_len.element_size() != 4 or b.alt_len.element_size() != 4:
            raise TypeError("allele_off must be int64, ref_len/alt_len 32-bit")
        n = b.n
        for t in (b.pos, b.allele_off, b.ref_len, b.alt_len):
            if t.numel() != n:
                raise ValueError("record arrays must all have n entries")
        if b.ext_id is not None and b.ext_id.numel() != n:
            raise ValueError("ext_id must have n entries")


_ENGINES: Dict[int, Engine] = {}


def default_engine(device=None) -> Engine:
    """Process-wide engine per device (GRCh38 table); ``AVDB_DEVICE=host`` (with no
    device given) selects the host-only engine of the per-call entries."""
    if device is None and os.environ.get("AVDB_DEVICE") == "host":
        device = "host"
    if device == "host":
        eng = _ENGINES.get("host")
        if eng is None:
            eng = _ENGINES["host"] = Engine("host")
        return eng
    N.require_gpu()
    idx = torch.cuda.current_device() if device is None else int(device)
    eng = _ENGINES.get(idx)
    if eng is None:
        eng = Engine(idx)
        _ENGINES[idx] = eng
    return eng
