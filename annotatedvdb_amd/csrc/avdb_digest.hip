// K4 — sha512t24u digests and the long-allele primary-key digest, gfx950.
//
// Long alleles (len(ref)+len(alt) > maxSequenceLength, primary_key_generator.py:53,110)
// are keyed chr:pos:<digest>[:refSNP] where the digest is GA4GH's computed
// identifier of the VRS Allele (compute_vrs_identifier :147-165):
// sha512t24u = base64url(SHA-512(blob)[0:24]).  Parity of the VRS blob layout is
// UNPINNED (vrs-python / SeqRepo are absent); the SHA-512 primitive is pinned
// against hashlib in tests.
//
// Pipeline for a batch:
//   k_long_hist     per-workgroup histogram of long records by SHA block count
//   k_long_scan     one workgroup: bucket-major exclusive scan -> offsets
//   k_long_scatter  list of long record indices, grouped by block count
//   k_vrs_digest    one lane per long record: SequenceLocation digest (2 blocks)
//                   then Allele digest, block-synchronously
// Grouping by block count keeps the 64 lanes of a wave on the same number of
// compressions.  Message words are built 8 bytes at a time: a word lying inside
// the ALT bytes is one funnel-shifted 8-byte heap load + byte swap; only the few
// words at segment boundaries are assembled bytewise.  The SHA-512 state and
// the 16-word schedule stay in registers; the compression has a single call
// site per kernel.
#include "avdb_fmt.hpp"  // ascii8 / ndigits (SWAR decimal text)

#include <vector>

namespace avdb {

__constant__ uint64_t K512[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

__constant__ uint64_t kIV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

__constant__ char kB64url[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

// VRS 1.x compact serialisations (keys sorted, no whitespace)
#define LOC0 "{\"interval\":{\"end\":{\"type\":\"Number\",\"value\":"
#define LOC1 "},\"start\":{\"type\":\"Number\",\"value\":"
#define LOC2 "},\"type\":\"SequenceInterval\"},\"sequence_id\":\""
#define LOC3 "\",\"type\":\"SequenceLocation\"}"
#define AL0 "{\"location\":\""
#define AL1 "\",\"state\":{\"sequence\":\""
#define AL2 "\",\"type\":\"LiteralSequenceExpression\"},\"type\":\"Allele\"}"
__constant__ char kLoc0[] = LOC0;
__constant__ char kLoc1[] = LOC1;
__constant__ char kLoc2[] = LOC2;
__constant__ char kLoc3[] = LOC3;
__constant__ char kAl0[] = AL0;
__constant__ char kAl1[] = AL1;
__constant__ char kAl2[] = AL2;
constexpr uint32_t nL0 = sizeof(LOC0) - 1;
constexpr uint32_t nL1 = sizeof(LOC1) - 1;
constexpr uint32_t nL2 = sizeof(LOC2) - 1;
constexpr uint32_t nL3 = sizeof(LOC3) - 1;
constexpr uint32_t nA0 = sizeof(AL0) - 1;
constexpr uint32_t nA1 = sizeof(AL1) - 1;
constexpr uint32_t nA2 = sizeof(AL2) - 1;
constexpr uint32_t kAlPrefix = nA0 + AVDB_DIGEST_CHARS + nA1;  // ALT starts here
static_assert(kAlPrefix == 68, "allele prefix");

// (kLongBuckets, long_bucket, long_code: avdb_internal.hpp)
static_assert(kAlPrefix + nA2 == kVrsAlleleFixedBytes, "VRS Allele message length");
constexpr int kCompactGrid = 2048;  // 8 workgroups per CU for the streaming passes

__device__ __forceinline__ uint32_t sha_blocks(uint64_t msg_bytes) {
  return uint32_t((msg_bytes + 17 + 127) / 128);
}

__device__ __forceinline__ uint32_t allele_blocks(uint32_t a) {
  return sha_blocks(uint64_t(kAlPrefix) + a + nA2);
}

// 64-bit rotate right by a constant as two 32-bit funnel shifts (v_alignbit_b32),
// instead of two 64-bit shifts and an or
template <int N>
__device__ __forceinline__ uint64_t rotr(uint64_t x) {
  const uint32_t lo = uint32_t(x), hi = uint32_t(x >> 32);
  uint32_t nlo, nhi;
  if constexpr (N < 32) {
    nlo = __builtin_amdgcn_alignbit(hi, lo, N);
    nhi = __builtin_amdgcn_alignbit(lo, hi, N);
  } else {
    nlo = __builtin_amdgcn_alignbit(lo, hi, N - 32);
    nhi = __builtin_amdgcn_alignbit(hi, lo, N - 32);
  }
  return (uint64_t(nhi) << 32) | nlo;
}

// gfx950 v_bitop3_b32: any 3-input bitwise function in one instruction per
// 32-bit half (truth table over inputs 0xF0, 0xCC, 0xAA).  xor3 folds the three
// rotations of Sigma/sigma, and Ch / Maj are single selects.
constexpr unsigned kXor3 = 0x96;  // x ^ y ^ z
constexpr unsigned kCh = 0xCA;    // x ? y : z
constexpr unsigned kMaj = 0xE8;   // majority(x, y, z)
template <unsigned LUT>
__device__ __forceinline__ uint64_t bop3(uint64_t x, uint64_t y, uint64_t z) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32(uint32_t(x), uint32_t(y), uint32_t(z), LUT);
  const uint32_t hi =
      __builtin_amdgcn_bitop3_b32(uint32_t(x >> 32), uint32_t(y >> 32), uint32_t(z >> 32), LUT);
  return (uint64_t(hi) << 32) | lo;
}

// 64-bit logical shift right by a constant: one v_lshrrev_b64 (the compiler
// splits x >> N into a funnel shift + a 32-bit shift; one instruction per sigma
// of the message schedule fewer: K4 2.39 -> 2.34 ms on C4k, k4_ab/r06_shr64_ab.txt)
template <int N>
__device__ __forceinline__ uint64_t shr(uint64_t x) {
  uint64_t r;
  asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "n"(N), "v"(x));
  return r;
}

// 64-bit add as one v_lshl_add_u64.  Written as inline asm because operands
// assembled from two 32-bit halves (bop3 results) are otherwise split by the
// compiler into a 64-bit add of the low half plus a 32-bit add of the high
// halves and register moves (~5 extra instructions per round).
__device__ __forceinline__ uint64_t add64(uint64_t x, uint64_t y) {
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

template <bool SCHED>
__device__ __forceinline__ void sha512_16(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t& e,
                                          uint64_t& f, uint64_t& g, uint64_t& hh, uint64_t* w, int r) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint64_t wt;
    if constexpr (!SCHED) {
      wt = w[j];
    } else {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = bop3<kXor3>(rotr<1>(w15), rotr<8>(w15), shr<7>(w15));
      const uint64_t s1 = bop3<kXor3>(rotr<19>(w2), rotr<61>(w2), shr<6>(w2));
      wt = add64(add64(w[j], w[(j + 9) & 15]), add64(s0, s1));
      w[j] = wt;
    }
    // hh + K + w does not depend on this round's e/a: off the critical path
    const uint64_t hkw = hh + (K512[r + j] + wt);
    const uint64_t S1 = bop3<kXor3>(rotr<14>(e), rotr<18>(e), rotr<41>(e));
    const uint64_t t1 = add64(hkw, add64(S1, bop3<kCh>(e, f, g)));
    const uint64_t S0 = bop3<kXor3>(rotr<28>(a), rotr<34>(a), rotr<39>(a));
    const uint64_t mj = bop3<kMaj>(a, b, c);
    hh = g; g = f; f = e; e = add64(d, t1); d = c; c = b; b = a; a = add64(t1, add64(S0, mj));
  }
}

// One SHA-512 compression; state and schedule in registers.  The first 16
// rounds (message words as given) are peeled off the scheduled 64.
__device__ __forceinline__ void sha512_block(uint64_t* H, uint64_t* w) {
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], hh = H[7];
  sha512_16<false>(a, b, c, d, e, f, g, hh, w, 0);
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) sha512_16<true>(a, b, c, d, e, f, g, hh, w, r);
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += hh;
}

// SHA padding byte at message position q for a message of T bytes in nb blocks
__device__ __forceinline__ uint8_t pad_byte(uint64_t q, uint64_t T, uint32_t nb) {
  if (q == T) return 0x80;
  const uint64_t end = uint64_t(nb) * 128;
  if (q >= end - 8) return uint8_t((T * 8) >> (8 * (end - 1 - q)));
  return 0;
}

// base64url of the first 24 digest bytes, packed as 4 little-endian words of chars
__device__ __forceinline__ void t24u_words(const uint64_t* H, uint64_t* out) {
#pragma unroll
  for (int o = 0; o < 4; ++o) out[o] = 0;
#pragma unroll
  for (int g = 0; g < 8; ++g) {  // 3 digest bytes -> 4 chars
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = 3 * g + k;
      v = (v << 8) | uint32_t((H[i >> 3] >> (56 - 8 * (i & 7))) & 0xFF);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int ci = 4 * g + k;
      const uint64_t ch = uint64_t(uint8_t(kB64url[(v >> (18 - 6 * k)) & 63]));
      out[ci >> 3] |= ch << (8 * (ci & 7));
    }
  }
}

__device__ __forceinline__ uint8_t word_char(const uint64_t* w4, uint32_t k) {  // k < 32
  const uint32_t q = k >> 3;
  const uint64_t x = q == 0 ? w4[0] : q == 1 ? w4[1] : q == 2 ? w4[2] : w4[3];
  return uint8_t(x >> (8 * (k & 7)));
}



__device__ __forceinline__ void store_digest(char* o, const uint64_t* cw) {
  if ((reinterpret_cast<uintptr_t>(o) & 7) == 0) {
    uint64_t* dst = reinterpret_cast<uint64_t*>(o);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = cw[k];
  } else {
    for (uint32_t k = 0; k < 32; ++k) o[k] = char(word_char(cw, k));
  }
}

// ---------------------------------------------------------------------------
// generic sha512t24u over caller byte strings
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sha512t24u(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, size_t n,
                                                       char* __restrict__ out) {
  // wide loads are only used for 8 bytes wholly inside a string, so both
  // aligned words they touch hold string bytes: unbounded heap is safe here
  const Heap hp{reinterpret_cast<uintptr_t>(data), ~uintptr_t(0)};
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t o = off[i];
    const uint64_t T = len[i];
    const uint32_t nb = sha_blocks(T);
    uint64_t H[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) H[k] = kIV[k];
    for (uint32_t b = 0; b < nb; ++b) {
      uint64_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint64_t p = uint64_t(b) * 128 + 8 * j;
        if (p + 8 <= T) {
          w[j] = __builtin_bswap64(heap_u64(hp, o + p));
        } else {
          uint64_t x = 0;
          for (int k = 0; k < 8; ++k) {
            const uint64_t q = p + k;
            const uint8_t by = q < T ? data[o + q] : pad_byte(q, T, nb);
            x = (x << 8) | by;
          }
          w[j] = x;
        }
      }
      sha512_block(H, w);
    }
    uint64_t cw[4];
    t24u_words(H, cw);
    store_digest(out + i * AVDB_DIGEST_CHARS, cw);
  }
}

// ---------------------------------------------------------------------------
// long-record list, grouped by allele-message block count (deterministic
// bucket-major layout: no contended atomics)
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool is_long_rec(uint32_t r, uint32_t a, uint32_t max_len) {
  return uint64_t(r) + a > max_len;
}

__device__ __forceinline__ uint32_t bucket_of(uint32_t a) { return long_bucket(a); }

// f(i, ref_len, alt_len) for every record of this workgroup's contiguous chunk;
// 4 records per lane per step through 16-byte loads when VEC (the chunk size is
// a multiple of 4, so the loads are aligned when the arrays are)
template <bool VEC, class F>
__device__ __forceinline__ void for_chunk_records(const uint32_t* __restrict__ rl,
                                                  const uint32_t* __restrict__ al, size_t n, F f) {
  const size_t per = (((n + gridDim.x - 1) / gridDim.x) + 3) & ~size_t(3);
  const size_t i0 = size_t(blockIdx.x) * per;
  const size_t i1 = i0 + per < n ? i0 + per : n;
  if constexpr (VEC) {
    // two groups per lane per step, both loaded before either is used
    const size_t step = 4 * size_t(blockDim.x);
    for (size_t j = i0 + 4 * size_t(threadIdx.x); j < i1; j += 2 * step) {
      const size_t j2 = j + step;
      u32x4 r0{}, a0{}, r1{}, a1{};
      const bool full0 = j + 4 <= i1, full1 = j2 + 4 <= i1;
      if (full0) {
        r0 = *reinterpret_cast<const u32x4*>(rl + j);
        a0 = *reinterpret_cast<const u32x4*>(al + j);
      }
      if (full1) {
        r1 = *reinterpret_cast<const u32x4*>(rl + j2);
        a1 = *reinterpret_cast<const u32x4*>(al + j2);
      }
      if (full0) {
        f(j, r0.x, a0.x);
        f(j + 1, r0.y, a0.y);
        f(j + 2, r0.z, a0.z);
        f(j + 3, r0.w, a0.w);
      } else {
        for (size_t k = j; k < i1; ++k) f(k, rl[k], al[k]);
      }
      if (full1) {
        f(j2, r1.x, a1.x);
        f(j2 + 1, r1.y, a1.y);
        f(j2 + 2, r1.z, a1.z);
        f(j2 + 3, r1.w, a1.w);
      } else {
        for (size_t k = j2; k < i1; ++k) f(k, rl[k], al[k]);
      }
    }
  } else {
    for (size_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) f(i, rl[i], al[i]);
  }
}

template <bool VEC>
__global__ __launch_bounds__(kBlock) void k_long_hist(const uint32_t* __restrict__ rl,
                                                      const uint32_t* __restrict__ al, size_t n,
                                                      uint32_t max_len, uint8_t* __restrict__ is_long,
                                                      uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_cnt[kLongBuckets];
  if (threadIdx.x < kLongBuckets) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  // (VEC: the four is_long bytes of a group leave as one 32-bit store)
  uint32_t flags = 0;
  for_chunk_records<VEC>(rl, al, n, [&](size_t i, uint32_t r, uint32_t a) {
    const bool lg = is_long_rec(r, a, max_len);
    if (VEC && is_long) {
      flags |= uint32_t(lg) << (8 * (i & 3));
      if ((i & 3) == 3) {
        *reinterpret_cast<uint32_t*>(is_long + (i - 3)) = flags;
        flags = 0;
      }
    } else if (is_long) {
      is_long[i] = lg;
    }
    if (lg) atomicAdd(&s_cnt[bucket_of(a)], 1u);
  });
  if (VEC && is_long) {  // a chunk ending inside a group (n % 4 != 0): its lane stores the rest
    const size_t per = (((n + gridDim.x - 1) / gridDim.x) + 3) & ~size_t(3);
    const size_t i0 = size_t(blockIdx.x) * per;
    const size_t i1 = i0 + per < n ? i0 + per : n;
    const size_t jt = i1 & ~size_t(3);
    if ((i1 & 3) && jt >= i0 && ((jt - i0) / 4) % blockDim.x == threadIdx.x)
      for (size_t k = jt; k < i1; ++k) is_long[k] = uint8_t(flags >> (8 * (k & 3)));
  }
  __syncthreads();
  if (threadIdx.x < kLongBuckets) counts[threadIdx.x * gridDim.x + blockIdx.x] = s_cnt[threadIdx.x];
}

// exclusive scan of the kLongBuckets * kCompactGrid counts by one 1024-thread
// workgroup: wave w owns a contiguous 1/16 of the array and reads it coalesced
// (lane l takes 16-byte word l of every 256-count step), all loads issued first
constexpr uint32_t kScanN = kLongBuckets * kCompactGrid;
constexpr uint32_t kScanSteps = kScanN / 16 / 256;
static_assert(kScanN % (16 * 256) == 0, "k_long_scan layout");

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = __lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, kWave);
    if (lane >= d) v += u;
  }
  return v;
}

__global__ __launch_bounds__(1024) void k_long_scan(uint32_t* __restrict__ counts,
                                                    unsigned int* __restrict__ total) {
  __shared__ uint32_t s_wave[16];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  u32x4* seg = reinterpret_cast<u32x4*>(counts + size_t(wv) * (kScanN / 16));
  u32x4 v[kScanSteps];
#pragma unroll
  for (uint32_t k = 0; k < kScanSteps; ++k) v[k] = seg[k * 64 + lane];
  uint32_t tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanSteps; ++k) tot += v[k].x + v[k].y + v[k].z + v[k].w;
  const uint32_t wsum = __shfl(wave_incl_scan(tot), 63, kWave);
  if (lane == 0) s_wave[wv] = wsum;
  __syncthreads();
  uint32_t base = 0;
  for (uint32_t w = 0; w < wv; ++w) base += s_wave[w];
#pragma unroll
  for (uint32_t k = 0; k < kScanSteps; ++k) {
    const uint32_t ls = v[k].x + v[k].y + v[k].z + v[k].w;
    const uint32_t incl = wave_incl_scan(ls);
    uint32_t run = base + incl - ls;
    u32x4 o;
    o.x = run; run += v[k].x;
    o.y = run; run += v[k].y;
    o.z = run; run += v[k].z;
    o.w = run;
    seg[k * 64 + lane] = o;
    base += __shfl(incl, 63, kWave);
  }
  if (threadIdx.x == 1023) *total = base;
}

// the same scatter from the is_long flags k_long_hist wrote (1 byte per record,
// 4 per load) instead of both length arrays (8 bytes per record): only a long
// record's ALT length is read again, for its bucket
__global__ __launch_bounds__(kBlock) void k_long_scatter_flags(const uint8_t* __restrict__ is_long,
                                                               const uint32_t* __restrict__ al, size_t n,
                                                               const uint32_t* __restrict__ offs,
                                                               uint32_t* __restrict__ list) {
  __shared__ uint32_t s_cur[kLongBuckets];
  if (threadIdx.x < kLongBuckets) s_cur[threadIdx.x] = offs[threadIdx.x * gridDim.x + blockIdx.x];
  __syncthreads();
  const size_t per = (((n + gridDim.x - 1) / gridDim.x) + 3) & ~size_t(3);  // k_long_hist's chunks
  const size_t i0 = size_t(blockIdx.x) * per;
  const size_t i1 = i0 + per < n ? i0 + per : n;
  const size_t step = 4 * size_t(blockDim.x);
  for (size_t j = i0 + 4 * size_t(threadIdx.x); j < i1; j += 2 * step) {
    const size_t j2 = j + step;
    const uint32_t f0 = j + 4 <= i1 ? *reinterpret_cast<const uint32_t*>(is_long + j) : 0u;
    const uint32_t f1 = j2 + 4 <= i1 ? *reinterpret_cast<const uint32_t*>(is_long + j2) : 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if ((f0 >> (8 * k)) & 1u) list[atomicAdd(&s_cur[bucket_of(al[j + k])], 1u)] = uint32_t(j + k);
      if ((f1 >> (8 * k)) & 1u) list[atomicAdd(&s_cur[bucket_of(al[j2 + k])], 1u)] = uint32_t(j2 + k);
    }
    // a chunk ending inside a group
    if (j + 4 > i1)
      for (size_t k = j; k < i1; ++k)
        if (is_long[k]) list[atomicAdd(&s_cur[bucket_of(al[k])], 1u)] = uint32_t(k);
    if (j2 < i1 && j2 + 4 > i1)
      for (size_t k = j2; k < i1; ++k)
        if (is_long[k]) list[atomicAdd(&s_cur[bucket_of(al[k])], 1u)] = uint32_t(k);
  }
}

// The keyed K2 already classified every record (long_code: 0 or 1 + bucket, one
// byte per record in the workspace): the histogram reads those bytes (1 B per
// record instead of both lengths, 8 B) and writes the is_long flags from them
__global__ __launch_bounds__(kBlock) void k_long_hist_codes(const uint8_t* __restrict__ codes, size_t n,
                                                            uint8_t* __restrict__ is_long,
                                                            uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_cnt[kLongBuckets];
  if (threadIdx.x < kLongBuckets) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const size_t per = (((n + gridDim.x - 1) / gridDim.x) + 3) & ~size_t(3);  // k_long_hist's chunks
  const size_t i0 = size_t(blockIdx.x) * per;
  const size_t i1 = i0 + per < n ? i0 + per : n;
  for (size_t j = i0 + 4 * size_t(threadIdx.x); j < i1; j += 4 * size_t(blockDim.x)) {
    if (j + 4 <= i1) {
      const uint32_t c4 = *reinterpret_cast<const uint32_t*>(codes + j);
      uint32_t f = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t c = (c4 >> (8 * k)) & 0xFFu;
        if (c) {
          f |= 1u << (8 * k);
          atomicAdd(&s_cnt[c - 1], 1u);
        }
      }
      if (is_long) *reinterpret_cast<uint32_t*>(is_long + j) = f;
    } else {
      for (size_t k = j; k < i1; ++k) {
        const uint32_t c = codes[k];
        if (c) atomicAdd(&s_cnt[c - 1], 1u);
        if (is_long) is_long[k] = c ? 1 : 0;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < kLongBuckets) counts[threadIdx.x * gridDim.x + blockIdx.x] = s_cnt[threadIdx.x];
}

// the scatter over the same chunks, buckets from the codes (no length reads)
__global__ __launch_bounds__(kBlock) void k_long_scatter_codes(const uint8_t* __restrict__ codes, size_t n,
                                                               const uint32_t* __restrict__ offs,
                                                               uint32_t* __restrict__ list) {
  __shared__ uint32_t s_cur[kLongBuckets];
  if (threadIdx.x < kLongBuckets) s_cur[threadIdx.x] = offs[threadIdx.x * gridDim.x + blockIdx.x];
  __syncthreads();
  const size_t per = (((n + gridDim.x - 1) / gridDim.x) + 3) & ~size_t(3);
  const size_t i0 = size_t(blockIdx.x) * per;
  const size_t i1 = i0 + per < n ? i0 + per : n;
  for (size_t j = i0 + 4 * size_t(threadIdx.x); j < i1; j += 4 * size_t(blockDim.x)) {
    const uint32_t c4 = j + 4 <= i1 ? *reinterpret_cast<const uint32_t*>(codes + j) : 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t c = (c4 >> (8 * k)) & 0xFFu;
      if (c) list[atomicAdd(&s_cur[c - 1], 1u)] = uint32_t(j + k);
    }
    if (j + 4 > i1)
      for (size_t k = j; k < i1; ++k)
        if (codes[k]) list[atomicAdd(&s_cur[codes[k] - 1], 1u)] = uint32_t(k);
  }
}

template <bool VEC>
__global__ __launch_bounds__(kBlock) void k_long_scatter(const uint32_t* __restrict__ rl,
                                                         const uint32_t* __restrict__ al, size_t n,
                                                         uint32_t max_len,
                                                         const uint32_t* __restrict__ offs,
                                                         uint32_t* __restrict__ list) {
  __shared__ uint32_t s_cur[kLongBuckets];
  if (threadIdx.x < kLongBuckets) s_cur[threadIdx.x] = offs[threadIdx.x * gridDim.x + blockIdx.x];
  __syncthreads();
  for_chunk_records<VEC>(rl, al, n, [&](size_t i, uint32_t r, uint32_t a) {
    if (is_long_rec(r, a, max_len)) list[atomicAdd(&s_cur[bucket_of(a)], 1u)] = uint32_t(i);
  });
}

// ---------------------------------------------------------------------------
// VRS Allele digest per long record
// ---------------------------------------------------------------------------
// Message words of one 128-byte block, produced by appending <= 8 bytes at a
// time (little-endian in a 64-bit accumulator); the words of block `blk` go to
// this lane's LDS slot as the big-endian values SHA-512 consumes.
struct MsgSink {
  uint64_t* slot;  // [word][lane]
  uint32_t jlo;    // first word of the block being built
  uint32_t j = 0;  // index of the word being filled
  uint32_t k = 0;  // bytes pending in w
  uint64_t w = 0;
  __device__ __forceinline__ MsgSink(uint64_t* sl, uint32_t blk) : slot(sl), jlo(16 * blk) {}
  __device__ __forceinline__ void word(uint64_t v) {  // v: the big-endian word value
    if (j - jlo < 16u) slot[(j - jlo) * kBlock] = v;
    ++j;
  }
  __device__ __forceinline__ void append(uint64_t x, uint32_t t) {  // 1 <= t <= 8
    w |= x << (8 * k);
    if (k + t >= 8) {
      word(__builtin_bswap64(w));
      w = k ? x >> (64 - 8 * k) : 0ull;
      k = k + t - 8;
    } else {
      k += t;
    }
  }
  // (string literals: the length and the chunks fold at compile time)
  __device__ __forceinline__ void lit(const char* s) {
    uint32_t n = 0;
    while (s[n]) ++n;
    for (uint32_t i = 0; i < n; i += 8) {
      const uint32_t t = n - i < 8u ? n - i : 8u;
      uint64_t x = 0;
      for (uint32_t q = 0; q < t; ++q) x |= uint64_t(uint8_t(s[i + q])) << (8 * q);
      append(x, t);
    }
  }
  __device__ __forceinline__ void digits(uint32_t v) {  // decimal, no leading zeros (SWAR, K7's dec_text)
    const Dec d = dec_text(v);
    append(d.lo, d.n < 8 ? d.n : 8);
    if (d.n > 8) append(d.hi, d.n - 8);
  }
  // SHA padding for a T-byte message of nb blocks: 0x80, zeros, 128-bit length
  __device__ __forceinline__ void finish(uint64_t T, uint32_t nb) {
    append(0x80, 1);
    if (k) {
      word(__builtin_bswap64(w));
      w = 0;
      k = 0;
    }
    const uint32_t last = nb * 16 - 1;
    while (j < last - 1) word(0);
    word(0);
    word(T * 8);
  }
};

// the VRS SequenceLocation serialisation of interval (S, E] on a contig whose 32
// refget chars are dig (4 little-endian words): its first block.  The
// serialisation is 183 + nE + nS bytes (2 SHA blocks for every 32-bit position)
// and the digits end at byte 79 + nE + nS < 128, so block 0 is complete once the
// digest chars are appended, and block 1 depends only on the contig and
// nE + nS: it is read from the table avdb_ctx_set_sequence_digests builds
// (location_tail_table) instead of being serialised again per record.
__device__ __forceinline__ void location_block0(uint64_t* slot, uint32_t S, uint32_t E, const uint64_t* dig) {
  MsgSink m(slot, 0);
  m.lit(LOC0);
  m.digits(E);
  m.lit(LOC1);
  m.digits(S);
  m.lit(LOC2);
#pragma unroll
  for (int q = 0; q < 4; ++q) m.append(dig[q], 8);
}

// compile-time little-endian 8-byte chunk of a string literal (zero past its end)
template <size_t N>
__device__ __forceinline__ uint64_t lit_word(const char (&s)[N], int at) {
  uint64_t x = 0;
  for (int q = 0; q < 8; ++q)
    if (at + q >= 0 && at + q < int(N) - 1) x |= uint64_t(uint8_t(s[at + q])) << (8 * q);
  return x;
}

// prefix bytes [8K, 8K+8) of the Allele message (those below kAlPrefix), little-endian
template <int K>
__device__ __forceinline__ uint64_t prefix_word(const uint64_t* locw) {
  constexpr int p = 8 * K, c_lo = int(nA0), c_hi = int(nA0) + AVDB_DIGEST_CHARS;
  uint64_t le = lit_word(AL0, p) | lit_word(AL1, p - c_hi);
  constexpr int c0 = p > c_lo ? p : c_lo, c1 = p + 8 < c_hi ? p + 8 : c_hi;
  if constexpr (c0 < c1) {
    constexpr int ci = c0 - c_lo, wi = ci >> 3, bo = ci & 7;
    uint64_t x = locw[wi] >> (8 * bo);
    if constexpr (bo != 0 && wi + 1 < 4) x |= locw[wi + 1] << (64 - 8 * bo);
    le |= (x & low_bytes_mask(uint32_t(c1 - c0))) << (8 * (c0 - p));
  }
  if constexpr (p + 8 > int(kAlPrefix)) le &= low_bytes_mask(uint32_t(int(kAlPrefix) - p));
  return le;
}

// The Allele serialisation AL0 + <32 location chars> + AL1 + ALT + AL2, then SHA
// padding: the 16 big-endian message words of block `ab` (uniform across the
// wave: lanes are grouped by block count), built in registers with no branch
// on the lane's ALT length.  A word is the OR of three masked sources:
//   prefix  words 0..8 of block 0 (literals + the location chars; static j)
//   ALT     one unaligned 8-byte heap load, masked to the bytes before Q
//   suffix  an 8-byte window of (8 zero bytes | AL2 | 0x80 | zeros) read from
//           the LDS table s_suf at the word's offset from Q (clamped: the
//           windows outside the suffix are zero)
// and the final block's last word is the message length in bits.
constexpr int kSufTab = 72;  // windows at offsets -8 .. 63 from the suffix start
// ALT word j of a block: 8 heap bytes from `at`.  CLAMP (a block reaching past
// the heap end): the load starts at most at the last 8 heap bytes and is shifted
// down (bytes past the heap end lie past the ALT and are masked off anyway).
template <bool CLAMP>
__device__ __forceinline__ uint64_t alt_word(const Heap& hp, uint64_t at) {
  if constexpr (!CLAMP) {
    return reinterpret_cast<g_u64u>(hp.lo + at)->v;
  } else {
    const uint64_t lim = (hp.hi - hp.lo) - 8;
    const uint64_t c = at < lim ? at : lim;
    const uint64_t y = reinterpret_cast<g_u64u>(hp.lo + c)->v;
    return at - c >= 8 ? 0ull : y >> (8 * (at - c));
  }
}

template <bool CLAMP>
__device__ __forceinline__ void allele_words(uint64_t* w, uint32_t ab, const uint64_t* locw, const Heap& hp,
                                             uint64_t altoff, int64_t Q, const uint64_t* s_suf) {
  const bool FIRST = ab == 0;  // uniform across the wave
  // word j's ALT bytes start at heap byte altoff + 128*ab + 8j - 68 (one base per
  // block, immediate offsets); bytes past the ALT are loaded and masked off
  const uint64_t b0 = altoff + 128 * uint64_t(ab) - kAlPrefix;  // ab >= 1: >= altoff + 60
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int64_t p = int64_t(ab) * 128 + 8 * j;  // first message byte of the word
    uint64_t le = 0;
    if (FIRST && j <= 8) {
      switch (j) {
        case 0: le = prefix_word<0>(locw); break;
        case 1: le = prefix_word<1>(locw); break;
        case 2: le = prefix_word<2>(locw); break;
        case 3: le = prefix_word<3>(locw); break;
        case 4: le = prefix_word<4>(locw); break;
        case 5: le = prefix_word<5>(locw); break;
        case 6: le = prefix_word<6>(locw); break;
        case 7: le = prefix_word<7>(locw); break;
        case 8: le = prefix_word<8>(locw); break;
        default: break;
      }
    }
    if (!FIRST || j >= 8) {
      // block 0 word 8: prefix bytes 64..67, then ALT bytes 0..3
      const uint64_t x = (FIRST && j == 8) ? alt_word<CLAMP>(hp, altoff) << 32 : alt_word<CLAMP>(hp, b0 + 8 * j);
      const int64_t nbytes = Q - p;  // ALT bytes from the word start (<= 0: none)
      le |= nbytes >= 8 ? x : (nbytes > 0 ? x & low_bytes_mask(uint32_t(nbytes)) : 0ull);
    }
    int64_t t = p - Q + 8;
    t = t < 0 ? 0 : (t > kSufTab - 1 ? kSufTab - 1 : t);
    le |= s_suf[t];
    w[j] = __builtin_bswap64(le);
  }
}

__device__ __forceinline__ void allele_block(uint64_t* w, uint32_t ab, const uint64_t* locw, const Heap& hp,
                                             uint64_t altoff, uint32_t a, uint64_t TA, uint32_t nb,
                                             const uint64_t* s_suf) {
  const int64_t Q = int64_t(kAlPrefix) + a;  // first suffix byte
  // a block wholly inside the ALT bytes for every lane of the wave (lanes are
  // grouped by block count, so all but the last two blocks of a long ALT are):
  // each word is one heap load, byte-swapped — no prefix, mask or suffix window
  const bool inside = ab >= 1 && int64_t(ab) * 128 + 128 <= Q;
  if (__all(inside)) {
    const uint64_t b0 = altoff + 128 * uint64_t(ab) - kAlPrefix;
    if (hp.lo + b0 + 128 <= hp.hi) {
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = __builtin_bswap64(alt_word<false>(hp, b0 + 8 * j));
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = __builtin_bswap64(alt_word<true>(hp, b0 + 8 * j));
    }
    return;
  }
  if (hp.lo + altoff + 128 * uint64_t(ab) + 128 <= hp.hi)
    allele_words<false>(w, ab, locw, hp, altoff, Q, s_suf);
  else
    allele_words<true>(w, ab, locw, hp, altoff, Q, s_suf);
  if (ab + 1 == nb) w[15] = TA * 8;  // (w[14], the high length word, is 0 from the table)
}

constexpr uint32_t kLocTailS = 19;  // nE + nS = 2..20

// Host: block 1 of every contig's SequenceLocation serialisation for each digit
// count nE + nS, as the big-endian message words SHA-512 consumes (the digit
// values lie in block 0; block 1 = the rest of LOC2, the digest chars, LOC3, the
// padding and the bit length 8 * (183 + nE + nS)).
void location_tail_table(const char* digests, int n_chrom, std::vector<uint64_t>& out) {
  out.assign(size_t(n_chrom) * kLocTailS * 16, 0);
  for (int c = 0; c < n_chrom; ++c) {
    for (uint32_t s = 2; s <= 20; ++s) {
      uint8_t m[256] = {0};
      size_t k = 0;
      auto put = [&](const char* t, size_t n) { for (size_t q = 0; q < n; ++q) m[k++] = uint8_t(t[q]); };
      put(LOC0, nL0);
      for (uint32_t q = 0; q < s; ++q) m[k++] = '0';  // E and S digits: their values lie in block 0
      put(LOC1, nL1);
      put(LOC2, nL2);
      put(digests + size_t(c) * AVDB_DIGEST_CHARS, AVDB_DIGEST_CHARS);
      put(LOC3, nL3);
      const uint64_t T = k;  // 183 + s
      m[k] = 0x80;
      for (int q = 0; q < 8; ++q) m[255 - q] = uint8_t((T * 8) >> (8 * q));
      uint64_t* o = &out[(size_t(c) * kLocTailS + (s - 2)) * 16];
      for (int j = 0; j < 16; ++j) {
        uint64_t v = 0;
        for (int q = 0; q < 8; ++q) v = (v << 8) | m[128 + 8 * j + q];
        o[j] = v;
      }
    }
  }
}

// Waves per SIMD (launch bound and persistent grid).  3: <= 168 VGPRs, no
// spills; the SHA-512 chains are latency-bound, so occupancy feeds the VALU.
#ifndef AVDB_DIGEST_WAVES
#define AVDB_DIGEST_WAVES 3
#endif
constexpr int kDigestWavesPerSimd = AVDB_DIGEST_WAVES;
// Optional second destination (avdb_vrs_digest_keys): the 32 characters also go
// straight into the primary-key text a deferred K7 / avdb_keyed_prep laid out
// (state AVDB_KEY_DIGEST_PENDING), at key_off[i] + len("label:pos:") — the fill
// pass's work, done where chrom / pos are already in registers (the separate
// pass re-read state, chrom, pos and key_off for every record: 0.43 ms on C4k).
struct KeyFill {
  const uint64_t* key_off;
  uint8_t* key_out;
  uint8_t* state;
};
__global__ __launch_bounds__(kBlock, kDigestWavesPerSimd) void k_vrs_digest(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ rl,
    const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap, size_t heap_bytes,
    const uint32_t* __restrict__ list, const unsigned int* __restrict__ count,
    const char* __restrict__ seq_digest, const uint64_t* __restrict__ loc_tail, int n_chrom,
    char* __restrict__ out, KeyFill F) {
  __shared__ uint64_t s_w[16 * kBlock];
  __shared__ uint64_t s_suf[kSufTab];
  if (threadIdx.x < kSufTab) {  // 8-byte windows of (8 zero bytes | AL2 | 0x80 | zeros)
    uint64_t x = 0;
    for (int q = 0; q < 8; ++q) {
      const int z = int(threadIdx.x) + q - 8;  // suffix byte index
      const uint32_t by = (z >= 0 && z < int(nA2)) ? uint8_t(kAl2[z]) : (z == int(nA2) ? 0x80u : 0u);
      x |= uint64_t(by) << (8 * q);
    }
    s_suf[threadIdx.x] = x;
  }
  __syncthreads();
  const Heap hp = make_heap(heap, heap_bytes);
  const unsigned int cnt = *count;
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (size_t t = size_t(blockIdx.x) * blockDim.x + threadIdx.x; t < cnt; t += stride) {
    const uint32_t i = list[t];
    const uint32_t c = chrom[i];
    const uint32_t r = rl[i], a = al[i];
    char* o = out + size_t(i) * AVDB_DIGEST_CHARS;
    if (c >= uint32_t(n_chrom)) {
      for (int k = 0; k < AVDB_DIGEST_CHARS; ++k) o[k] = '?';
      continue;
    }
    // gnomAD chr-pos-ref-alt -> interbase interval (pos-1, pos-1+len(ref)]
    const uint32_t S = pos[i] - 1u, E = S + r;
    const uint32_t nES = ndigits(E) + ndigits(S);  // 2..20
    constexpr uint32_t nbL = 2;  // sha_blocks(183 + nES) for every 32-bit position
    const uint64_t* tail = loc_tail + (size_t(c) * kLocTailS + (nES - 2)) * 16;
    const uint64_t* dg = reinterpret_cast<const uint64_t*>(seq_digest + size_t(c) * AVDB_DIGEST_CHARS);
    const uint64_t dig[4] = {dg[0], dg[1], dg[2], dg[3]};
    const uint64_t altoff = off[i] + r;
    const uint64_t TA = uint64_t(kAlPrefix) + a + nA2;
    const uint32_t nbA = sha_blocks(TA);
    uint64_t H[8], locw[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) H[k] = kIV[k];
    uint64_t* slot = &s_w[threadIdx.x];  // this lane's 16 message words, [word][lane]
    // One compression site (code size): SequenceLocation blocks take their
    // words from this lane's LDS slot, Allele blocks build them in registers;
    // b is uniform across the wave, so the branch does not diverge.
    for (uint32_t b = 0; b < nbL + nbA; ++b) {
      uint64_t w[16];
      if (b == 0) {
        location_block0(slot, S, E, dig);
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = slot[j * kBlock];
      } else if (b == 1) {
        const u32x4* t4 = reinterpret_cast<const u32x4*>(tail);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const u32x4 v = t4[j];
          w[2 * j] = uint64_t(v.x) | (uint64_t(v.y) << 32);
          w[2 * j + 1] = uint64_t(v.z) | (uint64_t(v.w) << 32);
        }
      } else {
        allele_block(w, b - nbL, locw, hp, altoff, a, TA, nbA, s_suf);
      }
      sha512_block(H, w);
      if (b + 1 == nbL) {  // location digest done: its chars feed the Allele blob
        t24u_words(H, locw);
#pragma unroll
        for (int k = 0; k < 8; ++k) H[k] = kIV[k];
      }
    }
    uint64_t cw[4];
    t24u_words(H, cw);
    store_digest(o, cw);
    if (F.key_out) {
      const uint8_t st = F.state[i];
      if ((st & 0x0Fu) == AVDB_KEY_DIGEST_PENDING) {
        gw_u64u q = reinterpret_cast<gw_u64u>((gbyte*)F.key_out + F.key_off[i] + key_body_at(c, pos[i]));
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k].v = cw[k];
        F.state[i] = uint8_t((st & 0xF0u) | AVDB_KEY_OK);
      }
    }
  }
}

}  // namespace avdb

using namespace avdb;

extern "C" int avdb_sha512t24u(avdb_ctx* ctx, const uint8_t* data, const uint64_t* off,
                               const uint32_t* len, size_t n, char* out, void* stream) {
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  if (n == 0) return AVDB_OK;
  if (!data || !off || !len || !out) { avdb_set_error("avdb_sha512t24u: null array"); return AVDB_EINVAL; }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  const unsigned grid = stream_grid(n, kBlock, 4096);
  hipLaunchKernelGGL(k_sha512t24u, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     data, off, len, n, out);
  AVDB_LAUNCH_CHECK("k_sha512t24u");
  return AVDB_OK;
}

// workspace: 256 (total) | counts u32[kLongBuckets * kCompactGrid] | list u32[n]
// | codes u8[n] (the keyed K2's long_code per record)
extern "C" int avdb_vrs_digest_workspace_size(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = 256 + 4 * size_t(kLongBuckets) * kCompactGrid + 4 * n + ((n + 15) & ~size_t(15));
  return AVDB_OK;
}

namespace avdb {
uint8_t* vrs_long_codes_of(void* workspace, size_t n) {
  return static_cast<uint8_t*>(workspace) + 256 + 4 * size_t(kLongBuckets) * kCompactGrid + 4 * n;
}
}  // namespace avdb

extern "C" int avdb_vrs_digest(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                               const uint64_t* allele_off, const uint32_t* ref_len,
                               const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                               size_t n, uint32_t max_seq_len, void* workspace,
                               size_t workspace_bytes, char* digest_out, uint8_t* is_long,
                               void* stream) {
  return avdb_vrs_digest_ex(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, n, max_seq_len,
                            workspace, workspace_bytes, digest_out, is_long, 0u, stream);
}

static int vrs_digest_impl(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                           const uint64_t* allele_off, const uint32_t* ref_len,
                           const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                           size_t n, uint32_t max_seq_len, void* workspace,
                           size_t workspace_bytes, char* digest_out, uint8_t* is_long,
                           uint32_t flags, KeyFill fill, void* stream) {
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  if (n == 0) return AVDB_OK;
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap || !digest_out) {
    avdb_set_error("avdb_vrs_digest: null array");
    return AVDB_EINVAL;
  }
  if (!ctx->has_digests || !ctx->d_seq_digest || !ctx->d_loc_tail) {
    avdb_set_error("avdb_vrs_digest: sequence digests not set (avdb_ctx_set_sequence_digests)");
    return AVDB_EINVAL;
  }
  if (n >= 0xFFFFFFFFull) { avdb_set_error("avdb_vrs_digest: n must be < 2^32"); return AVDB_EINVAL; }
  size_t need = 0;
  avdb_vrs_digest_workspace_size(n, &need);
  if (!workspace || workspace_bytes < need) {
    avdb_set_error("avdb_vrs_digest: workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  if (reinterpret_cast<uintptr_t>(workspace) % 16) {
    avdb_set_error("avdb_vrs_digest: workspace must be 16-byte aligned");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* total = static_cast<unsigned int*>(workspace);
  auto* counts = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + 256);
  auto* list = counts + size_t(kLongBuckets) * kCompactGrid;
  const bool vec = (reinterpret_cast<uintptr_t>(ref_len) | reinterpret_cast<uintptr_t>(alt_len)) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(is_long) % 4 == 0;
  const bool codes_ready = (flags & AVDB_DIGEST_CODES_READY) && reinterpret_cast<uintptr_t>(is_long) % 4 == 0;
  const uint8_t* codes = vrs_long_codes_of(workspace, n);
  if (codes_ready)
    hipLaunchKernelGGL(k_long_hist_codes, dim3(kCompactGrid), dim3(kBlock), 0, s, codes, n, is_long, counts);
  else if (vec)
    hipLaunchKernelGGL(k_long_hist<true>, dim3(kCompactGrid), dim3(kBlock), 0, s, ref_len, alt_len, n,
                       max_seq_len, is_long, counts);
  else
    hipLaunchKernelGGL(k_long_hist<false>, dim3(kCompactGrid), dim3(kBlock), 0, s, ref_len, alt_len, n,
                       max_seq_len, is_long, counts);
  AVDB_LAUNCH_CHECK("k_long_hist");
  hipLaunchKernelGGL(k_long_scan, dim3(1), dim3(1024), 0, s, counts, total);
  AVDB_LAUNCH_CHECK("k_long_scan");
  if (codes_ready)
    hipLaunchKernelGGL(k_long_scatter_codes, dim3(kCompactGrid), dim3(kBlock), 0, s, codes, n, counts, list);
  else if (vec && is_long)
    hipLaunchKernelGGL(k_long_scatter_flags, dim3(kCompactGrid), dim3(kBlock), 0, s, is_long, alt_len, n, counts,
                       list);
  else if (vec)
    hipLaunchKernelGGL(k_long_scatter<true>, dim3(kCompactGrid), dim3(kBlock), 0, s, ref_len, alt_len, n,
                       max_seq_len, counts, list);
  else
    hipLaunchKernelGGL(k_long_scatter<false>, dim3(kCompactGrid), dim3(kBlock), 0, s, ref_len, alt_len, n,
                       max_seq_len, counts, list);
  AVDB_LAUNCH_CHECK("k_long_scatter");
  // persistent grid over the grouped list
  // (a smaller grid leaves CUs to K7 running beside it: avdb_ctx_set_option)
  const int per_cu = ctx->k4_blocks_per_cu < kDigestWavesPerSimd ? ctx->k4_blocks_per_cu : kDigestWavesPerSimd;
  const unsigned grid = ctx->k4_grid > 0 ? unsigned(ctx->k4_grid) : unsigned(ctx->n_cu * per_cu);
  hipLaunchKernelGGL(k_vrs_digest, dim3(grid), dim3(kBlock), 0, s, chrom, pos,
                     allele_off,
                     ref_len, alt_len, heap, heap_bytes, list, total, ctx->d_seq_digest, ctx->d_loc_tail,
                     ctx->tab.n, digest_out, fill);
  AVDB_LAUNCH_CHECK("k_vrs_digest");
  return AVDB_OK;
}

extern "C" int avdb_vrs_digest_ex(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                  const uint64_t* allele_off, const uint32_t* ref_len,
                                  const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                                  size_t n, uint32_t max_seq_len, void* workspace,
                                  size_t workspace_bytes, char* digest_out, uint8_t* is_long,
                                  uint32_t flags, void* stream) {
  return vrs_digest_impl(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, n, max_seq_len, workspace,
                         workspace_bytes, digest_out, is_long, flags, KeyFill{nullptr, nullptr, nullptr}, stream);
}

extern "C" int avdb_vrs_digest_keys(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                    const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                                    const uint8_t* heap, size_t heap_bytes, size_t n, uint32_t max_seq_len,
                                    void* workspace, size_t workspace_bytes, char* digest_out, uint8_t* is_long,
                                    uint32_t flags, const uint64_t* key_off, uint8_t* key_out, uint8_t* key_state,
                                    void* stream) {
  if (!key_off || !key_out || !key_state) {
    avdb_set_error("avdb_vrs_digest_keys: null key text");
    return AVDB_EINVAL;
  }
  return vrs_digest_impl(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, n, max_seq_len, workspace,
                         workspace_bytes, digest_out, is_long, flags, KeyFill{key_off, key_out, key_state}, stream);
}
