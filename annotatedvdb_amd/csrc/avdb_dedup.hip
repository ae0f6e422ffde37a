// K3 pk_dedup — in-batch primary-key deduplication, gfx950.
//
// The key is chr:pos:ref:alt[:refSNP] (primary_key_generator.py:99-122; the
// long-allele form swaps ref:alt for a digest of (chr,pos,ref,alt)), so two
// records share a key iff (chrom, pos, ref bytes, alt bytes, ext_id) are equal.
// The reference never dedups within a batch — COPY inserts duplicates and
// Load/lib/sql/annotatedvdb_schema/patches/removeDuplicates.sql:2-24 removes
// them after the fact; the contract here is keep-first-occurrence, stable order.
//
// grouped path: equal (chrom,pos) records are contiguous (position-sorted VCF),
//   so each record only looks back over its own (chrom,pos) run.
// hash path: 64-bit fingerprints, an open-addressing table that keeps the
//   minimum record index per fingerprint (atomicMin), then a byte-exact compare
//   against the winner; a fingerprint collision falls back to an exact scan.
// Allele bytes are compared / hashed 8 bytes per load (Heap helpers).
#include "avdb_internal.hpp"

namespace avdb {

__device__ __forceinline__ bool same_record(const Heap& h, const uint64_t* __restrict__ off,
                                            const uint32_t* __restrict__ rl,
                                            const uint32_t* __restrict__ al,
                                            const uint64_t* __restrict__ ext, size_t i, size_t j) {
  const uint32_t r = rl[i], a = al[i];
  if (rl[j] != r || al[j] != a) return false;
  if (ext && ext[i] != ext[j]) return false;
  return heap_equal(h, off[i], off[j], r + a);
}

// Byte compares longer than this run wave-cooperatively (64 lanes x 8 bytes per
// step) instead of serially in one lane.
constexpr uint32_t kCoopBytes = 64;

// Whole-wave equality test of L bytes at heap offsets p and q (all lanes call
// with the same arguments; returns the same answer in every lane).
__device__ __forceinline__ bool wave_heap_equal(const Heap& h, uint64_t p, uint64_t q, uint32_t L) {
  const uint32_t lane = __lane_id();
  for (uint32_t base = 0; base < L; base += 8 * kWave) {
    const uint32_t k = base + 8 * lane;
    bool diff = false;
    if (k < L) {
      const uint64_t m = low_bytes_mask(L - k);
      diff = ((heap_u64(h, p + k) ^ heap_u64(h, q + k)) & m) != 0;
    }
    if (__ballot(diff)) return false;
  }
  return true;
}

// Keep bit of record i: the nearest earlier record of its (chrom,pos) run with
// the same lengths and external id is compared; short candidates in-lane, long
// ones queued for the whole wave.  Earlier run members are scanned in order, so
// the first equal one decides (keep-first).  scan == false (record i-1 is known
// to be outside the run) skips the scan.  Every lane of the wave must call it
// together (ballots).
__device__ __forceinline__ uint8_t dedup_record(const Heap& h, const uint8_t* __restrict__ chrom,
                                                const uint32_t* __restrict__ pos,
                                                const uint64_t* __restrict__ off,
                                                const uint32_t* __restrict__ rl,
                                                const uint32_t* __restrict__ al,
                                                const uint64_t* __restrict__ ext, size_t i, bool live,
                                                bool scan) {
  uint8_t k = 1;
  size_t j = i;
  uint32_t L = 0;
  bool pending = false;
  if (live && scan) {
    const uint8_t c = chrom[i];
    const uint32_t p = pos[i];
    const uint32_t r = rl[i], a = al[i];
    const uint64_t e = ext ? ext[i] : 0;
    L = r + a;
    while (j-- > 0) {
      if (chrom[j] != c || pos[j] != p) break;
      if (rl[j] != r || al[j] != a || (ext && ext[j] != e)) continue;
      if (L > kCoopBytes) { pending = true; break; }
      if (heap_equal(h, off[i], off[j], L)) { k = 0; break; }
    }
  }
  // long candidates: one cooperative compare per queued lane; a mismatch sends
  // that lane on to its next candidate (rare: equal lengths at one position)
  uint64_t q = __ballot(pending);
  while (q) {
    const int l = __ffsll((unsigned long long)q) - 1;
    const uint64_t pi = __shfl(live ? off[i] : 0ull, l, kWave);
    const uint64_t pj = __shfl(pending ? off[j] : 0ull, l, kWave);
    const uint32_t Ll = __shfl(L, l, kWave);
    const bool eq = wave_heap_equal(h, pi, pj, Ll);
    if (__lane_id() == l) {
      if (eq) {
        k = 0;
        pending = false;
      } else {  // continue this lane's scan past j
        pending = false;
        const uint8_t c = chrom[i];
        const uint32_t p = pos[i];
        const uint32_t r = rl[i], a = al[i];
        const uint64_t e = ext ? ext[i] : 0;
        while (j-- > 0) {
          if (chrom[j] != c || pos[j] != p) break;
          if (rl[j] != r || al[j] != a || (ext && ext[j] != e)) continue;
          pending = true;
          break;
        }
      }
    }
    q = __ballot(pending);
  }
  return k;
}

__device__ __forceinline__ void count_dups(uint32_t dups, unsigned long long* g_ctr) {
  if (!g_ctr) return;
  for (int d = 32; d > 0; d >>= 1) dups += __shfl_down(dups, d, kWave);
  if (__lane_id() == 0 && dups) atomicAdd(&g_ctr[AVDB_CTR_DUPLICATES], (unsigned long long)dups);
}

__global__ __launch_bounds__(kBlock) void k_dedup_grouped(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ rl,
    const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap, size_t heap_bytes,
    const uint64_t* __restrict__ ext, size_t n, uint8_t* __restrict__ keep,
    unsigned long long* __restrict__ g_ctr) {
  const Heap h = make_heap(heap, heap_bytes);
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  uint32_t dups = 0;
  // wave-uniform trip count so every lane reaches the cooperative compares
  for (size_t base = size_t(blockIdx.x) * blockDim.x; base < n; base += stride) {
    const size_t i = base + threadIdx.x;
    const bool live = i < n;
    const uint8_t k = dedup_record(h, chrom, pos, off, rl, al, ext, i, live, true);
    if (live) {
      keep[i] = k;
      dups += 1u - k;
    }
  }
  count_dups(dups, g_ctr);
}

// Vector form (aligned arrays): 4 consecutive records per lane from 16-byte
// loads.  A record whose predecessor (same lane, the previous lane via a
// shuffle, or one load for lane 0) has another (chrom,pos) is kept without
// touching memory again — the common case; the rest go through dedup_record.
__global__ __launch_bounds__(kBlock) void k_dedup_grouped4(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ rl,
    const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap, size_t heap_bytes,
    const uint64_t* __restrict__ ext, size_t n, uint8_t* __restrict__ keep,
    unsigned long long* __restrict__ g_ctr) {
  const Heap h = make_heap(heap, heap_bytes);
  const size_t ngroups = (n + 3) / 4;
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  uint32_t dups = 0;
  for (size_t base = size_t(blockIdx.x) * blockDim.x; base < ngroups; base += stride) {
    const size_t g = base + threadIdx.x;
    const size_t i0 = 4 * g;
    const bool full = i0 + 4 <= n;
    uint32_t c4 = 0;
    u32x4 p4{};
    if (full) {
      c4 = *reinterpret_cast<const uint32_t*>(chrom + i0);
      p4 = *reinterpret_cast<const u32x4*>(pos + i0);
    } else if (i0 < n) {
      for (uint32_t t = 0; t < 4 && i0 + t < n; ++t) {
        c4 |= uint32_t(chrom[i0 + t]) << (8 * t);
        p4[t] = pos[i0 + t];
      }
    }
    // predecessor of record i0: the previous lane's last record, or a load
    uint32_t pc = __shfl_up(c4 >> 24, 1, kWave), pp = __shfl_up(p4.w, 1, kWave);
    if (__lane_id() == 0 && i0 > 0 && i0 - 1 < n) {
      pc = chrom[i0 - 1];
      pp = pos[i0 - 1];
    }
    bool same[4];
    same[0] = i0 > 0 && (c4 & 0xFFu) == pc && p4.x == pp;
    same[1] = ((c4 >> 8) & 0xFFu) == (c4 & 0xFFu) && p4.y == p4.x;
    same[2] = ((c4 >> 16) & 0xFFu) == ((c4 >> 8) & 0xFFu) && p4.z == p4.y;
    same[3] = (c4 >> 24) == ((c4 >> 16) & 0xFFu) && p4.w == p4.z;
    uint32_t k4 = 0x01010101u;
    const bool any = i0 < n && (same[0] || same[1] || same[2] || same[3]);
    if (__ballot(any)) {
      // The usual case: the record equals its immediate predecessor.  All four
      // records' lengths / ids / offsets (and the predecessor's) are loaded at
      // once and the short byte compares issued together; a record the
      // predecessor does not settle goes through dedup_record below.
      uint32_t r[5] = {0, 0, 0, 0, 0}, a[5] = {0, 0, 0, 0, 0};
      uint64_t e[5] = {0, 0, 0, 0, 0}, o[5] = {0, 0, 0, 0, 0};
      if (any) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const size_t i = i0 + t < n ? i0 + t : n - 1;
          r[t + 1] = rl[i];
          a[t + 1] = al[i];
          e[t + 1] = ext ? ext[i] : 0;
          o[t + 1] = off[i];
        }
        if (same[0]) {
          r[0] = rl[i0 - 1];
          a[0] = al[i0 - 1];
          e[0] = ext ? ext[i0 - 1] : 0;
          o[0] = off[i0 - 1];
        }
      }
      uint32_t unresolved = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (!(any && same[t] && i0 + t < n)) continue;
        const uint32_t L = r[t + 1] + a[t + 1];
        if (r[t + 1] == r[t] && a[t + 1] == a[t] && e[t + 1] == e[t] && L <= kCoopBytes &&
            heap_equal(h, o[t + 1], o[t], L))
          k4 &= ~(1u << (8 * t));
        else
          unresolved |= 1u << t;
      }
      if (__ballot(unresolved != 0)) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const size_t i = i0 + t;
          const bool live = i < n;
          const uint8_t k =
              dedup_record(h, chrom, pos, off, rl, al, ext, i, live, live && ((unresolved >> t) & 1u));
          if (!k) k4 &= ~(1u << (8 * t));
        }
      }
    }
    if (full) {
      *reinterpret_cast<uint32_t*>(keep + i0) = k4;
      dups += 4u - __popc(k4);
    } else {
      for (uint32_t t = 0; t < 4 && i0 + t < n; ++t) {
        const uint8_t k = uint8_t((k4 >> (8 * t)) & 1u);
        keep[i0 + t] = k;
        dups += 1u - k;
      }
    }
  }
  count_dups(dups, g_ctr);
}

// Two-phase grouped dedup (aligned arrays + a workspace of kListHead + 4n bytes).
// Phase A streams chrom/pos 4 records per lane, writes keep = 1 for every
// record, and lists the records that share their predecessor's (chrom,pos) —
// the only ones that can repeat an earlier key.  Each workgroup owns a
// contiguous chunk of groups and lists its suspects in its own slice of the
// list (one LDS atomic per wave; a single device-wide counter serialises at
// ~90 atomics/us, which cost 1 ms here).  Phase B runs the same workgroup
// count: workgroup b gives each of its chunk's suspects a lane of its own for
// the run scan, so a suspect's dependent memory round trips are paid once per
// 64 suspects instead of once per wave of mostly unique records.
constexpr int kListGridMax = 4096;
constexpr size_t kListHead = 4 * kListGridMax;  // per-workgroup suspect counts
static_assert(kListHead == kDedupListHead && unsigned(kListGridMax) == kDedupMaxGroups, "K3 list layout");

__device__ __forceinline__ void chunk_of(size_t items, size_t* lo, size_t* hi) {
  const size_t per = (items + gridDim.x - 1) / gridDim.x;
  const size_t a = size_t(blockIdx.x) * per;
  *lo = a < items ? a : items;
  *hi = a + per < items ? a + per : items;
}

__global__ __launch_bounds__(kBlock) void k_dedup_mark4(const uint8_t* __restrict__ chrom,
                                                        const uint32_t* __restrict__ pos, size_t n,
                                                        uint8_t* __restrict__ keep,
                                                        uint32_t* __restrict__ counts,
                                                        uint32_t* __restrict__ list) {
  __shared__ uint32_t s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  size_t g0, g1;
  chunk_of((n + 3) / 4, &g0, &g1);
  uint32_t* mine = list + 4 * g0;
  for (size_t base = g0; base < g1; base += blockDim.x) {
    const size_t g = base + threadIdx.x;
    const size_t i0 = 4 * g;
    const bool live = g < g1;
    const bool full = live && i0 + 4 <= n;
    uint32_t c4 = 0;
    u32x4 p4{};
    if (full) {
      c4 = *reinterpret_cast<const uint32_t*>(chrom + i0);
      p4 = *reinterpret_cast<const u32x4*>(pos + i0);
    } else if (live) {
      for (uint32_t t = 0; t < 4 && i0 + t < n; ++t) {
        c4 |= uint32_t(chrom[i0 + t]) << (8 * t);
        p4[t] = pos[i0 + t];
      }
    }
    uint32_t pc = __shfl_up(c4 >> 24, 1, kWave), pp = __shfl_up(p4.w, 1, kWave);
    if (__lane_id() == 0 && live && i0 > 0) {
      pc = chrom[i0 - 1];
      pp = pos[i0 - 1];
    }
    uint32_t same = 0;
    same |= uint32_t(i0 > 0 && (c4 & 0xFFu) == pc && p4.x == pp);
    same |= uint32_t(((c4 >> 8) & 0xFFu) == (c4 & 0xFFu) && p4.y == p4.x) << 1;
    same |= uint32_t(((c4 >> 16) & 0xFFu) == ((c4 >> 8) & 0xFFu) && p4.z == p4.y) << 2;
    same |= uint32_t((c4 >> 24) == ((c4 >> 16) & 0xFFu) && p4.w == p4.z) << 3;
    if (!full) same &= (live && i0 < n) ? (1u << uint32_t(n - i0 < 4 ? n - i0 : 4)) - 1u : 0u;
    // wave-aggregated append of this lane's suspects to the workgroup's slice
    const uint32_t cnt = __popc(same);
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t u = __shfl_up(incl, d, kWave);
      if (__lane_id() >= d) incl += u;
    }
    const uint32_t total = __shfl(incl, kWave - 1, kWave);
    if (total) {
      uint32_t at = 0;
      if (__lane_id() == kWave - 1) at = atomicAdd(&s_cnt, total);
      at = __shfl(at, kWave - 1, kWave) + incl - cnt;
      for (uint32_t m = same; m; m &= m - 1) mine[at++] = uint32_t(i0 + __builtin_ctz(m));
    }
    if (full) {
      *reinterpret_cast<uint32_t*>(keep + i0) = 0x01010101u;
    } else if (live) {
      for (uint32_t t = 0; t < 4 && i0 + t < n; ++t) keep[i0 + t] = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = s_cnt;
}

__global__ __launch_bounds__(kBlock) void k_dedup_resolve_list(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ rl,
    const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap, size_t heap_bytes,
    const uint64_t* __restrict__ ext, size_t n, const uint32_t* __restrict__ counts,
    const uint32_t* __restrict__ list, uint8_t* __restrict__ keep, unsigned long long* __restrict__ g_ctr,
    size_t slice) {
  const Heap h = make_heap(heap, heap_bytes);
  size_t g0, g1;
  chunk_of((n + 3) / 4, &g0, &g1);
  // slice: the keyed K2 listed the suspects (one slice of `slice` entries per K2
  // workgroup, as many resolve workgroups); else k_dedup_mark4's chunks
  const uint32_t* mine = slice ? list + size_t(blockIdx.x) * slice : list + 4 * g0;
  const uint32_t cnt = counts[blockIdx.x];
  uint32_t dups = 0;
  // wave-uniform trip count (dedup_record's cooperative compares need the whole wave)
  for (uint32_t base = 0; base < cnt; base += blockDim.x) {
    const uint32_t t = base + threadIdx.x;
    const bool live = t < cnt;
    const size_t i = live ? mine[t] : 0;
    // A suspect shares (chrom, pos) with record i-1 (k_dedup_mark4).  The usual run
    // is two records, so i-1's lengths / id / offset and i-2's (chrom, pos) are
    // loaded together with i's, and a short compare against i-1 settles most
    // suspects in two dependent memory trips; dedup_record's serial look-back
    // (chrom / pos, then lengths, then bytes, per candidate) takes the rest.
    bool settled = false;
    uint8_t k = 1;
    if (live) {
      const uint32_t r = rl[i], a = al[i], r1 = rl[i - 1], a1 = al[i - 1];
      const uint64_t e = ext ? ext[i] : 0ull, e1 = ext ? ext[i - 1] : 0ull;
      const uint64_t o = off[i], o1 = off[i - 1];
      const bool run3 = i >= 2 && chrom[i - 2] == chrom[i] && pos[i - 2] == pos[i];
      const uint32_t L = r + a;
      const bool cand = r1 == r && a1 == a && e1 == e;
      if (cand && L <= kCoopBytes) {
        if (heap_equal(h, o, o1, L)) {
          k = 0;
          settled = true;
        } else {
          settled = !run3;
        }
      } else if (!cand) {
        settled = !run3;
      }
    }
    const uint8_t ks = dedup_record(h, chrom, pos, off, rl, al, ext, i, live, live && !settled);
    if (!settled) k = ks;
    if (live && !k) {
      keep[i] = 0;
      ++dups;
    }
  }
  count_dups(dups, g_ctr);
}

// 64-bit fingerprint of (chrom, pos, ext, ref_len, alt_len, bytes)
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ uint64_t fingerprint(const Heap& hp, uint64_t off, uint32_t r, uint32_t a,
                                                uint8_t c, uint32_t p, uint64_t e) {
  uint64_t h = mix64((uint64_t(c) << 32) ^ p ^ 0x9E3779B97F4A7C15ull);
  h = mix64(h ^ e);
  h = mix64(h ^ ((uint64_t(r) << 32) | a));
  const uint32_t L = r + a;
  for (uint32_t k = 0; k < L; k += 8) h = mix64(h ^ (heap_u64(hp, off + k) & low_bytes_mask(L - k)));
  return h ? h : 1ull;  // 0 marks an empty slot
}

__global__ __launch_bounds__(kBlock) void k_dedup_insert(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ rl,
    const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap, size_t heap_bytes,
    const uint64_t* __restrict__ ext, size_t n, uint64_t* __restrict__ fp,
    unsigned long long* __restrict__ tkey, uint32_t* __restrict__ tidx, uint64_t mask) {
  const Heap hp = make_heap(heap, heap_bytes);
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t h = fingerprint(hp, off[i], rl[i], al[i], chrom[i], pos[i], ext ? ext[i] : 0);
    fp[i] = h;
    uint64_t slot = mix64(h) & mask;
    for (;;) {  // table has >= 2n slots: always terminates
      const unsigned long long prev = atomicCAS(&tkey[slot], 0ull, (unsigned long long)h);
      if (prev == 0ull || prev == h) { atomicMin(&tidx[slot], uint32_t(i)); break; }
      slot = (slot + 1) & mask;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_dedup_resolve(
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ rl,
    const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap, size_t heap_bytes,
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ ext, size_t n, const uint64_t* __restrict__ fp,
    const unsigned long long* __restrict__ tkey, const uint32_t* __restrict__ tidx,
    uint64_t mask, uint8_t* __restrict__ keep, unsigned long long* __restrict__ g_ctr) {
  const Heap hp = make_heap(heap, heap_bytes);
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  uint32_t dups = 0, coll = 0;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t h = fp[i];
    uint64_t slot = mix64(h) & mask;
    while (tkey[slot] != h) slot = (slot + 1) & mask;
    const uint32_t w = tidx[slot];
    uint8_t k = 1;
    if (w != uint32_t(i)) {
      if (chrom[w] == chrom[i] && pos[w] == pos[i] && same_record(hp, off, rl, al, ext, i, w)) {
        k = 0;
      } else {
        // fingerprint collision with a different key: exact scan of earlier
        // records carrying the same fingerprint (astronomically rare)
        ++coll;
        for (size_t j = 0; j < i; ++j)
          if (fp[j] == h && chrom[j] == chrom[i] && pos[j] == pos[i] &&
              same_record(hp, off, rl, al, ext, i, j)) { k = 0; break; }
      }
    }
    keep[i] = k;
    dups += 1u - k;
  }
  if (g_ctr) {
    for (int d = 32; d > 0; d >>= 1) {
      dups += __shfl_down(dups, d, kWave);
      coll += __shfl_down(coll, d, kWave);
    }
    if (__lane_id() == 0) {
      if (dups) atomicAdd(&g_ctr[AVDB_CTR_DUPLICATES], (unsigned long long)dups);
      if (coll) atomicAdd(&g_ctr[AVDB_CTR_HASH_COLLISIONS], (unsigned long long)coll);
    }
  }
}

}  // namespace avdb

using namespace avdb;

static uint64_t table_slots(size_t n) {
  uint64_t s = 1024;
  while (s < 2ull * n) s <<= 1;
  return s;
}

extern "C" int avdb_pk_dedup_workspace_size(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  const uint64_t slots = table_slots(n);
  // fp[n] u64 | keys[slots] u64 | idx[slots] u32
  *bytes = size_t(8 * n + 8 * slots + 4 * slots + 256);
  return AVDB_OK;
}

extern "C" int avdb_pk_dedup_ex(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                                const uint8_t* heap, size_t heap_bytes, const uint64_t* ext_id, size_t n,
                                void* workspace, size_t workspace_bytes, uint8_t* keep, uint64_t* counters,
                                uint32_t flags, void* stream) {
  if (!(flags & AVDB_DEDUP_MARKED))
    return avdb_pk_dedup(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, ext_id, n, 1, workspace,
                         workspace_bytes, keep, counters, stream);
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  if (n == 0) return AVDB_OK;
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap || !keep || !workspace) {
    avdb_set_error("avdb_pk_dedup_ex: null array");
    return AVDB_EINVAL;
  }
  if (flags & ~uint32_t(AVDB_DEDUP_MARKED | AVDB_DEDUP_ONEPASS)) {
    avdb_set_error("avdb_pk_dedup_ex: unknown flags 0x%x", flags);
    return AVDB_EINVAL;
  }
  unsigned grid = 0;
  size_t slice = 0;
  if (flags & AVDB_DEDUP_ONEPASS) keyed_onepass_dd_layout(n, &grid, &slice);
  else keyed_prep_layout(ctx, n, &grid, &slice);
  if (!grid || workspace_bytes < kListHead + 4 * size_t(grid) * slice) {
    avdb_set_error("avdb_pk_dedup_ex: the workspace does not hold the keyed K2's suspect lists");
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  auto* counts = static_cast<uint32_t*>(workspace);
  auto* list = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + kListHead);
  hipLaunchKernelGGL(k_dedup_resolve_list, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), chrom,
                     pos, allele_off, ref_len, alt_len, heap, heap_bytes, ext_id, n, counts, list, keep,
                     reinterpret_cast<unsigned long long*>(counters), slice);
  AVDB_LAUNCH_CHECK("k_dedup_resolve_list");
  return AVDB_OK;
}

extern "C" int avdb_pk_dedup(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                             const uint64_t* allele_off, const uint32_t* ref_len,
                             const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                             const uint64_t* ext_id, size_t n, int grouped, void* workspace,
                             size_t workspace_bytes, uint8_t* keep, uint64_t* counters,
                             void* stream) {
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  if (n == 0) return AVDB_OK;
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap || !keep) {
    avdb_set_error("avdb_pk_dedup: null array");
    return AVDB_EINVAL;
  }
  if (n >= 0xFFFFFFFFull) { avdb_set_error("avdb_pk_dedup: n must be < 2^32"); return AVDB_EINVAL; }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* ctr = reinterpret_cast<unsigned long long*>(counters);
  const unsigned grid = stream_grid(n, kBlock * 4, 4096);
  if (grouped) {
    const bool vec = (reinterpret_cast<uintptr_t>(chrom) | reinterpret_cast<uintptr_t>(keep)) % 4 == 0 &&
                     reinterpret_cast<uintptr_t>(pos) % 16 == 0;
    const unsigned grid4 = stream_grid((n + 3) / 4, kBlock * 2, kListGridMax);
    // (the one-kernel run scan below measured 22.2 us against 5.7 + 7.6 us for the
    // list form on C1's 1.1 M records: the list form whenever a workspace is given)
    if (vec && workspace && workspace_bytes >= kListHead + 4 * ((n + 3) & ~size_t(3)) &&
        reinterpret_cast<uintptr_t>(workspace) % 16 == 0) {
      auto* counts = static_cast<uint32_t*>(workspace);
      auto* list = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + kListHead);
      hipLaunchKernelGGL(k_dedup_mark4, dim3(grid4), dim3(kBlock), 0, s, chrom, pos, n, keep, counts, list);
      AVDB_LAUNCH_CHECK("k_dedup_mark4");
      hipLaunchKernelGGL(k_dedup_resolve_list, dim3(grid4), dim3(kBlock), 0, s, chrom, pos, allele_off,
                         ref_len, alt_len, heap, heap_bytes, ext_id, n, counts, list, keep, ctr, size_t(0));
      AVDB_LAUNCH_CHECK("k_dedup_resolve_list");
    } else if (vec) {
      hipLaunchKernelGGL(k_dedup_grouped4, dim3(grid4), dim3(kBlock), 0, s, chrom, pos, allele_off,
                         ref_len, alt_len, heap, heap_bytes, ext_id, n, keep, ctr);
      AVDB_LAUNCH_CHECK("k_dedup_grouped4");
    } else {
      hipLaunchKernelGGL(k_dedup_grouped, dim3(grid), dim3(kBlock), 0, s, chrom, pos, allele_off,
                         ref_len, alt_len, heap, heap_bytes, ext_id, n, keep, ctr);
      AVDB_LAUNCH_CHECK("k_dedup_grouped");
    }
    return AVDB_OK;
  }
  size_t need = 0;
  avdb_pk_dedup_workspace_size(n, &need);
  if (!workspace || workspace_bytes < need) {
    avdb_set_error("avdb_pk_dedup: workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  const uint64_t slots = table_slots(n);
  char* w = static_cast<char*>(workspace);
  uint64_t* fp = reinterpret_cast<uint64_t*>(w);
  auto* tkey = reinterpret_cast<unsigned long long*>(w + 8 * n);
  uint32_t* tidx = reinterpret_cast<uint32_t*>(w + 8 * n + 8 * slots);
  AVDB_HIP_TRY(hipMemsetAsync(tkey, 0, 8 * slots, s));
  AVDB_HIP_TRY(hipMemsetAsync(tidx, 0xFF, 4 * slots, s));
  hipLaunchKernelGGL(k_dedup_insert, dim3(grid), dim3(kBlock), 0, s, chrom, pos, allele_off,
                     ref_len, alt_len, heap, heap_bytes, ext_id, n, fp, tkey, tidx, slots - 1);
  AVDB_LAUNCH_CHECK("k_dedup_insert");
  hipLaunchKernelGGL(k_dedup_resolve, dim3(grid), dim3(kBlock), 0, s, allele_off, ref_len,
                     alt_len, heap, heap_bytes, chrom, pos, ext_id, n, fp, tkey, tidx, slots - 1,
                     keep, ctr);
  AVDB_LAUNCH_CHECK("k_dedup_resolve");
  return AVDB_OK;
}
