// K6 — duplicate check against variants already in the database (gfx950).
//
// Replaces the per-variant database round trip of --skipExisting:
// VCFVariantLoader.__parse_alt_alleles -> is_duplicate(metaseq_id, returnMatch=True)
// (Util/lib/python/loaders/vcf_variant_loader.py:284-291, variant_loader.py:173-174)
// -> VariantRecord.exists -> SQL map_variants(id, firstHitOnly=True, checkAltVariants=True)
// (Util/lib/python/database/variant.py:41,287-309; the SQL itself is external).
// The rows already loaded are supplied once as a key set (their metaseq ids,
// e.g. exported with COPY ... TO); the batch is then a hash join on the device:
//   k_keyset_insert  one lane per key: streaming 64-bit hash of the key bytes,
//                    open addressing (atomicCAS on the hash, atomicMin on the key
//                    index: the first of equal keys wins = firstHitOnly)
//   k_keyset_probe   one lane per record: the same hash over the record's metaseq
//                    id "chrom:pos:ref:alt" generated on the fly (never
//                    materialised), byte-exact confirmation against the key; with
//                    check_alt, a miss retries "chrom:pos:alt:ref" (alleles switched)
#include "avdb_internal.hpp"

namespace avdb {

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// streaming hash of a byte sequence: bytes packed little-endian into 8-byte
// words, each completed word mixed in; the length closes it.  Keys and
// generated metaseq ids go through the same byte stream, so equal strings hash
// equal however they are assembled.
struct Hasher {
  uint64_t h = 0x9E3779B97F4A7C15ull, w = 0;
  uint32_t n = 0;
  __device__ __forceinline__ void put(uint32_t c) {
    w |= uint64_t(c & 0xFFu) << (8 * (n & 7));
    if ((++n & 7) == 0) { h = mix(h ^ w); w = 0; }
  }
  __device__ __forceinline__ uint64_t done() const {
    const uint64_t x = mix(h ^ w ^ (uint64_t(n) << 56));
    return x ? x : 1ull;  // 0 marks an empty slot
  }
};

// "chrom:pos:" of a record (<= 16 bytes); contig labels of chromosomes.py:9-38
__device__ __forceinline__ uint32_t metaseq_prefix(uint32_t c, uint32_t pos, uint8_t* b) {
  uint32_t k = 0;
  if (c < 22) {
    const uint32_t v = c + 1;
    if (v >= 10) b[k++] = uint8_t('0' + v / 10);
    b[k++] = uint8_t('0' + v % 10);
  } else {
    b[k++] = c == 22 ? 'X' : (c == 23 ? 'Y' : 'M');
  }
  b[k++] = ':';
  char t[10];
  int d = 0;
  do { t[d++] = char('0' + pos % 10u); pos /= 10u; } while (pos);
  while (d) b[k++] = uint8_t(t[--d]);
  b[k++] = ':';
  return k;
}

__device__ __forceinline__ uint64_t hash_record(const uint8_t* pre, uint32_t plen, const uint8_t* x,
                                                uint32_t xl, const uint8_t* y, uint32_t yl) {
  Hasher hs;
  for (uint32_t i = 0; i < plen; ++i) hs.put(pre[i]);
  for (uint32_t i = 0; i < xl; ++i) hs.put(x[i]);
  hs.put(':');
  for (uint32_t i = 0; i < yl; ++i) hs.put(y[i]);
  return hs.done();
}

// key bytes == pre + x + ':' + y ?
__device__ __forceinline__ bool key_equals(const uint8_t* key, uint64_t klen, const uint8_t* pre, uint32_t plen,
                                           const uint8_t* x, uint32_t xl, const uint8_t* y, uint32_t yl) {
  if (klen != uint64_t(plen) + xl + 1 + yl) return false;
  for (uint32_t i = 0; i < plen; ++i)
    if (key[i] != pre[i]) return false;
  key += plen;
  for (uint32_t i = 0; i < xl; ++i)
    if (key[i] != x[i]) return false;
  if (key[xl] != ':') return false;
  key += xl + 1;
  for (uint32_t i = 0; i < yl; ++i)
    if (key[i] != y[i]) return false;
  return true;
}

__global__ __launch_bounds__(kBlock) void k_keyset_insert(const uint8_t* __restrict__ keys,
                                                          const uint64_t* __restrict__ key_off, size_t n,
                                                          unsigned long long* __restrict__ tkey,
                                                          uint32_t* __restrict__ tidx, uint64_t mask) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    Hasher hs;
    for (uint64_t b = key_off[i]; b < key_off[i + 1]; ++b) hs.put(keys[b]);
    const uint64_t h = hs.done();
    uint64_t slot = mix(h ^ 0x5bd1e995ull) & mask;
    for (;;) {  // >= 2n slots: terminates
      const unsigned long long prev = atomicCAS(&tkey[slot], 0ull, (unsigned long long)h);
      if (prev == 0ull || prev == h) { atomicMin(&tidx[slot], uint32_t(i)); break; }
      slot = (slot + 1) & mask;
    }
  }
}

// first key equal to pre+x+':'+y, or -1; *coll counts 64-bit hash collisions
__device__ int32_t lookup(const uint8_t* keys, const uint64_t* key_off, size_t n_keys,
                          const unsigned long long* tkey, const uint32_t* tidx, uint64_t mask,
                          const uint8_t* pre, uint32_t plen, const uint8_t* x, uint32_t xl, const uint8_t* y,
                          uint32_t yl, uint32_t* coll) {
  const uint64_t h = hash_record(pre, plen, x, xl, y, yl);
  uint64_t slot = mix(h ^ 0x5bd1e995ull) & mask;
  for (;;) {
    const unsigned long long t = tkey[slot];
    if (t == 0ull) return -1;
    if (t == h) break;
    slot = (slot + 1) & mask;
  }
  const uint32_t k = tidx[slot];
  if (key_equals(keys + key_off[k], key_off[k + 1] - key_off[k], pre, plen, x, xl, y, yl)) return int32_t(k);
  // a different key with the same 64-bit hash (astronomically rare): exact scan
  ++*coll;
  for (size_t j = 0; j < n_keys; ++j)
    if (key_equals(keys + key_off[j], key_off[j + 1] - key_off[j], pre, plen, x, xl, y, yl)) return int32_t(j);
  return -1;
}

__global__ __launch_bounds__(kBlock) void k_keyset_probe(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, size_t n_keys,
    const unsigned long long* __restrict__ tkey, const uint32_t* __restrict__ tidx, uint64_t mask,
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ rl, const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap,
    size_t n, int check_alt, int32_t* __restrict__ match, uint8_t* __restrict__ kind,
    unsigned long long* __restrict__ g_ctr) {
  uint32_t hits = 0, coll = 0;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t c = chrom[i];
    int32_t m = -1;
    uint8_t kd = 0;
    if (c >= 25) {
      kd = AVDB_MATCH_HOST;  // no canonical label: the caller resolves it
    } else {
      uint8_t pre[16];
      const uint32_t plen = metaseq_prefix(c, pos[i], pre);
      const uint8_t* ref = heap + off[i];
      const uint8_t* alt = ref + rl[i];
      m = lookup(keys, key_off, n_keys, tkey, tidx, mask, pre, plen, ref, rl[i], alt, al[i], &coll);
      if (m >= 0) {
        kd = AVDB_MATCH_EXACT;
      } else if (check_alt) {
        m = lookup(keys, key_off, n_keys, tkey, tidx, mask, pre, plen, alt, al[i], ref, rl[i], &coll);
        if (m >= 0) kd = AVDB_MATCH_SWITCHED;
      }
    }
    match[i] = m;
    kind[i] = kd;
    hits += m >= 0;
  }
  if (g_ctr) {
    for (int d = 32; d > 0; d >>= 1) {
      hits += __shfl_down(hits, d, kWave);
      coll += __shfl_down(coll, d, kWave);
    }
    if (__lane_id() == 0) {
      if (hits) atomicAdd(&g_ctr[AVDB_CTR_EXISTING], (unsigned long long)hits);
      if (coll) atomicAdd(&g_ctr[AVDB_CTR_HASH_COLLISIONS], (unsigned long long)coll);
    }
  }
}

// K6 over arbitrary strings (e.g. the primary keys K7 rendered): one lane per
// query string q[q_off[i] .. q_off[i+1]) (skipped where skip[i] != 0);
// match[i] = index of the first equal key, or -1
__device__ __forceinline__ bool str_equals(const uint8_t* a, uint64_t alen, const uint8_t* b, uint64_t blen) {
  if (alen != blen) return false;
  for (uint64_t i = 0; i < alen; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

__global__ __launch_bounds__(kBlock) void k_keyset_probe_text(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, size_t n_keys,
    const unsigned long long* __restrict__ tkey, const uint32_t* __restrict__ tidx, uint64_t mask,
    const uint8_t* __restrict__ q, const uint64_t* __restrict__ q_off, const uint8_t* __restrict__ skip, size_t n,
    int32_t* __restrict__ match, unsigned long long* __restrict__ g_ctr) {
  uint32_t hits = 0, coll = 0;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    int32_t m = -1;
    if (!skip || !skip[i]) {
      const uint8_t* s = q + q_off[i];
      const uint64_t len = q_off[i + 1] - q_off[i];
      Hasher hs;
      for (uint64_t b = 0; b < len; ++b) hs.put(s[b]);
      const uint64_t h = hs.done();
      uint64_t slot = mix(h ^ 0x5bd1e995ull) & mask;
      for (;;) {
        const unsigned long long t = tkey[slot];
        if (t == 0ull) break;
        if (t == h) {
          const uint32_t k = tidx[slot];
          if (str_equals(keys + key_off[k], key_off[k + 1] - key_off[k], s, len)) {
            m = int32_t(k);
          } else {  // a different key with the same 64-bit hash: exact scan
            ++coll;
            for (size_t j = 0; j < n_keys && m < 0; ++j)
              if (str_equals(keys + key_off[j], key_off[j + 1] - key_off[j], s, len)) m = int32_t(j);
          }
          break;
        }
        slot = (slot + 1) & mask;
      }
    }
    match[i] = m;
    hits += m >= 0;
  }
  if (g_ctr) {
    for (int d = 32; d > 0; d >>= 1) {
      hits += __shfl_down(hits, d, kWave);
      coll += __shfl_down(coll, d, kWave);
    }
    if (__lane_id() == 0) {
      if (hits) atomicAdd(&g_ctr[AVDB_CTR_EXISTING], (unsigned long long)hits);
      if (coll) atomicAdd(&g_ctr[AVDB_CTR_HASH_COLLISIONS], (unsigned long long)coll);
    }
  }
}

}  // namespace avdb

using namespace avdb;

static uint64_t keyset_slots(size_t n) {
  uint64_t s = 1024;
  while (s < 2ull * n) s <<= 1;
  return s;
}

extern "C" int avdb_keyset_workspace_size(size_t n_keys, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  const uint64_t s = keyset_slots(n_keys);
  *bytes = s * 8 + s * 4;
  return AVDB_OK;
}

extern "C" int avdb_keyset_build(avdb_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, size_t n_keys,
                                 void* table, size_t table_bytes, void* stream) {
  if (!ctx || !key_off || !table || (n_keys && !keys)) {
    avdb_set_error("avdb_keyset_build: null argument");
    return AVDB_EINVAL;
  }
  if (n_keys >= 0x7FFFFFFFull) { avdb_set_error("avdb_keyset_build: too many keys"); return AVDB_EINVAL; }
  size_t need = 0;
  avdb_keyset_workspace_size(n_keys, &need);
  if (table_bytes < need) {
    avdb_set_error("avdb_keyset_build: table of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t slots = keyset_slots(n_keys);
  auto* tkey = static_cast<unsigned long long*>(table);
  auto* tidx = reinterpret_cast<uint32_t*>(tkey + slots);
  AVDB_HIP_TRY(hipMemsetAsync(tkey, 0, slots * 8, s));
  AVDB_HIP_TRY(hipMemsetAsync(tidx, 0xFF, slots * 4, s));
  if (n_keys == 0) return AVDB_OK;
  hipLaunchKernelGGL(k_keyset_insert, dim3(stream_grid(n_keys, kBlock, 4096)), dim3(kBlock), 0, s, keys, key_off,
                     n_keys, tkey, tidx, slots - 1);
  AVDB_LAUNCH_CHECK("k_keyset_insert");
  return AVDB_OK;
}

extern "C" int avdb_keyset_probe(avdb_ctx* ctx, const void* table, size_t table_bytes, const uint8_t* keys,
                                 const uint64_t* key_off, size_t n_keys, const uint8_t* chrom,
                                 const uint32_t* pos, const uint64_t* allele_off, const uint32_t* ref_len,
                                 const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes, size_t n,
                                 int check_alt, int32_t* match, uint8_t* kind, uint64_t* counters,
                                 void* stream) {
  (void)heap_bytes;
  if (!ctx || !table || !key_off || !match || !kind) {
    avdb_set_error("avdb_keyset_probe: null argument");
    return AVDB_EINVAL;
  }
  size_t need = 0;
  avdb_keyset_workspace_size(n_keys, &need);
  if (table_bytes < need) {
    avdb_set_error("avdb_keyset_probe: table of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  if (n == 0) return AVDB_OK;
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap) {
    avdb_set_error("avdb_keyset_probe: null record array");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  const uint64_t slots = keyset_slots(n_keys);
  auto* tkey = static_cast<const unsigned long long*>(table);
  auto* tidx = reinterpret_cast<const uint32_t*>(tkey + slots);
  hipLaunchKernelGGL(k_keyset_probe, dim3(stream_grid(n, kBlock, 4096)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), keys, key_off, n_keys, tkey, tidx, slots - 1, chrom, pos,
                     allele_off, ref_len, alt_len, heap, n, check_alt, match, kind,
                     reinterpret_cast<unsigned long long*>(counters));
  AVDB_LAUNCH_CHECK("k_keyset_probe");
  return AVDB_OK;
}

extern "C" int avdb_keyset_probe_text(avdb_ctx* ctx, const void* table, size_t table_bytes, const uint8_t* keys,
                                      const uint64_t* key_off, size_t n_keys, const uint8_t* q,
                                      const uint64_t* q_off, const uint8_t* skip, size_t n, int32_t* match,
                                      uint64_t* counters, void* stream) {
  if (!ctx || !table || !key_off || !match || (n && !q_off)) {
    avdb_set_error("avdb_keyset_probe_text: null argument");
    return AVDB_EINVAL;
  }
  size_t need = 0;
  avdb_keyset_workspace_size(n_keys, &need);
  if (table_bytes < need) {
    avdb_set_error("avdb_keyset_probe_text: table of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  if (n == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  const uint64_t slots = keyset_slots(n_keys);
  auto* tkey = static_cast<const unsigned long long*>(table);
  auto* tidx = reinterpret_cast<const uint32_t*>(tkey + slots);
  hipLaunchKernelGGL(k_keyset_probe_text, dim3(stream_grid(n, kBlock, 4096)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), keys, key_off, n_keys, tkey, tidx, slots - 1, q, q_off, skip,
                     n, match, reinterpret_cast<unsigned long long*>(counters));
  AVDB_LAUNCH_CHECK("k_keyset_probe_text");
  return AVDB_OK;
}
