// K4 — sha512t24u digests and the long-allele primary-key digest, gfx950.
//
// Long alleles (len(ref)+len(alt) > maxSequenceLength, primary_key_generator.py:53,110)
// are keyed chr:pos:<digest>[:refSNP] where the digest is GA4GH's computed
// identifier of the VRS Allele (compute_vrs_identifier :147-165):
// sha512t24u = base64url(SHA-512(blob)[0:24]).  Parity of the VRS blob layout is
// UNPINNED (vrs-python / SeqRepo are absent); the SHA-512 primitive is pinned
// against hashlib in tests.
//
// Long records are a few % of a batch, so they are first compacted with a
// wave ballot + one atomic per wave (k_long_compact), then hashed one record
// per lane by a persistent grid (k_vrs_digest).  Each lane's 128-byte SHA-512
// message block lives in LDS, laid out [word][lane] (conflict-free 8-byte
// accesses); the 80 rounds run in registers with a static-indexed schedule.
#include "avdb_internal.hpp"

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

__device__ __forceinline__ uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// SHA-512 compression of one 128-byte block.  Both the block (16 words) and
// the chaining state (8 words) live in LDS, [word][lane], so this single
// out-of-line copy needs no scratch and no struct pointer.
__device__ __noinline__ void sha512_compress(uint64_t* buf, uint64_t* hs) {
  uint64_t w[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = buf[t * kBlock];
  uint64_t a = hs[0], b = hs[kBlock], c = hs[2 * kBlock], d = hs[3 * kBlock];
  uint64_t e = hs[4 * kBlock], f = hs[5 * kBlock], g = hs[6 * kBlock], hh = hs[7 * kBlock];
#pragma unroll 1
  for (int r = 0; r < 80; r += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint64_t wt;
      if (r == 0) {
        wt = w[j];
      } else {
        const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
        const uint64_t s0 = rotr(w15, 1) ^ rotr(w15, 8) ^ (w15 >> 7);
        const uint64_t s1 = rotr(w2, 19) ^ rotr(w2, 61) ^ (w2 >> 6);
        wt = w[j] + s0 + w[(j + 9) & 15] + s1;
        w[j] = wt;
      }
      const uint64_t S1 = rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41);
      const uint64_t ch = (e & f) ^ (~e & g);
      const uint64_t t1 = hh + S1 + ch + K512[r + j] + wt;
      const uint64_t S0 = rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39);
      const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint64_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
  }
  hs[0] += a; hs[kBlock] += b; hs[2 * kBlock] += c; hs[3 * kBlock] += d;
  hs[4 * kBlock] += e; hs[5 * kBlock] += f; hs[6 * kBlock] += g; hs[7 * kBlock] += hh;
}

// Streaming byte feeder; acc/nb/widx/total stay in registers.
struct Sha512 {
  uint64_t acc;
  uint32_t nb;      // bytes in acc (0..7)
  uint32_t widx;    // words in block buffer (0..15)
  uint64_t total;   // message bytes
  uint64_t* buf;    // LDS: word w of this lane at buf[w * kBlock]
  uint64_t* hs;     // LDS: chaining word k of this lane at hs[k * kBlock]

  __device__ __forceinline__ void init(uint64_t* lds_buf, uint64_t* lds_h) {
    buf = lds_buf; hs = lds_h;
    hs[0] = 0x6a09e667f3bcc908ull; hs[kBlock] = 0xbb67ae8584caa73bull;
    hs[2 * kBlock] = 0x3c6ef372fe94f82bull; hs[3 * kBlock] = 0xa54ff53a5f1d36f1ull;
    hs[4 * kBlock] = 0x510e527fade682d1ull; hs[5 * kBlock] = 0x9b05688c2b3e6c1full;
    hs[6 * kBlock] = 0x1f83d9abfb41bd6bull; hs[7 * kBlock] = 0x5be0cd19137e2179ull;
    acc = 0; nb = 0; widx = 0; total = 0;
  }
  __device__ __forceinline__ void put_raw(uint8_t byte) {
    acc = (acc << 8) | byte;
    if (++nb == 8) {
      buf[widx * kBlock] = acc;
      acc = 0; nb = 0;
      if (++widx == 16) { sha512_compress(buf, hs); widx = 0; }
    }
  }
  __device__ __forceinline__ void put(uint8_t byte) { put_raw(byte); ++total; }
  __device__ __forceinline__ void put_str(const char* s, int n) { for (int i = 0; i < n; ++i) put(uint8_t(s[i])); }
  __device__ __forceinline__ void put_bytes(const uint8_t* s, uint32_t n) { for (uint32_t i = 0; i < n; ++i) put(s[i]); }
  __device__ __forceinline__ void put_u32_dec(uint32_t v) {
    uint32_t p10 = 1;
    while (v / p10 >= 10u) p10 *= 10u;
    for (; p10; p10 /= 10u) put(uint8_t('0' + (v / p10) % 10u));
  }
  __device__ __forceinline__ void finish() {
    const uint64_t bits = total * 8;
    put_raw(0x80);
    while (widx * 8 + nb != 112) put_raw(0);
    for (int i = 0; i < 8; ++i) put_raw(0);  // high 64 bits of the length
    for (int i = 7; i >= 0; --i) put_raw(uint8_t(bits >> (8 * i)));
  }
  __device__ __forceinline__ uint64_t h(int k) const { return hs[k * kBlock]; }
};

__constant__ char kB64url[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

// base64url of the first 24 digest bytes -> 32 chars
__device__ __forceinline__ void t24u(const Sha512& sh, char* out) {
  const uint64_t h0 = sh.h(0), h1 = sh.h(1), h2 = sh.h(2);
  uint8_t d[24];
#pragma unroll
  for (int i = 0; i < 24; ++i) {
    const uint64_t hw = i < 8 ? h0 : (i < 16 ? h1 : h2);
    d[i] = uint8_t(hw >> (56 - 8 * (i & 7)));
  }
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const uint32_t v = (uint32_t(d[3 * g]) << 16) | (uint32_t(d[3 * g + 1]) << 8) | d[3 * g + 2];
    out[4 * g + 0] = kB64url[(v >> 18) & 63];
    out[4 * g + 1] = kB64url[(v >> 12) & 63];
    out[4 * g + 2] = kB64url[(v >> 6) & 63];
    out[4 * g + 3] = kB64url[v & 63];
  }
}

__global__ __launch_bounds__(kBlock) void k_sha512t24u(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, size_t n,
                                                       char* __restrict__ out) {
  __shared__ uint64_t s_buf[16 * kBlock];
  __shared__ uint64_t s_h[8 * kBlock];
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    Sha512 sh;
    sh.init(&s_buf[threadIdx.x], &s_h[threadIdx.x]);
    sh.put_bytes(data + off[i], len[i]);
    sh.finish();
    t24u(sh, out + i * AVDB_DIGEST_CHARS);
  }
}

// compact indices of long records (wave ballot + one atomic per wave)
__global__ __launch_bounds__(kBlock) void k_long_compact(const uint32_t* __restrict__ rl,
                                                         const uint32_t* __restrict__ al, size_t n,
                                                         uint32_t max_len, uint8_t* __restrict__ is_long,
                                                         uint32_t* __restrict__ list,
                                                         unsigned int* __restrict__ count) {
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  const size_t base0 = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (size_t i = base0; i - threadIdx.x < n; i += stride) {  // wave-uniform trip count
    const bool live = i < n;
    const bool lg = live && (uint64_t(rl[i]) + al[i] > max_len);
    if (live && is_long) is_long[i] = lg;
    const uint64_t m = __ballot(lg);
    if (m) {
      const int lane = __lane_id();
      unsigned int base = 0;
      if (lane == 0) base = atomicAdd(count, (unsigned int)__popcll(m));
      base = __shfl(base, 0, kWave);
      if (lg) {
        const uint64_t below = lane ? (m << (64 - lane)) : 0ull;
        list[base + __popcll(below)] = uint32_t(i);
      }
    }
  }
}

__constant__ char kLoc0[] = "{\"interval\":{\"end\":{\"type\":\"Number\",\"value\":";
__constant__ char kLoc1[] = "},\"start\":{\"type\":\"Number\",\"value\":";
__constant__ char kLoc2[] = "},\"type\":\"SequenceInterval\"},\"sequence_id\":\"";
__constant__ char kLoc3[] = "\",\"type\":\"SequenceLocation\"}";
__constant__ char kAl0[] = "{\"location\":\"";
__constant__ char kAl1[] = "\",\"state\":{\"sequence\":\"";
__constant__ char kAl2[] = "\",\"type\":\"LiteralSequenceExpression\"},\"type\":\"Allele\"}";

__global__ __launch_bounds__(kBlock) void k_vrs_digest(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ rl,
    const uint32_t* __restrict__ al, const uint8_t* __restrict__ heap,
    const uint32_t* __restrict__ list, const unsigned int* __restrict__ count,
    const char* __restrict__ seq_digest, int n_chrom, char* __restrict__ out) {
  __shared__ uint64_t s_buf[16 * kBlock];
  __shared__ uint64_t s_h[8 * kBlock];
  const unsigned int cnt = *count;
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (size_t t = size_t(blockIdx.x) * blockDim.x + threadIdx.x; t < cnt; t += stride) {
    const uint32_t i = list[t];
    const uint32_t c = chrom[i];
    const uint32_t start = pos[i] - 1u;  // gnomAD chr-pos-ref-alt -> interbase (pos-1, pos-1+len(ref)]
    const uint32_t r = rl[i], a = al[i];
    char* o = out + size_t(i) * AVDB_DIGEST_CHARS;
    if (c >= uint32_t(n_chrom)) {
      for (int k = 0; k < AVDB_DIGEST_CHARS; ++k) o[k] = '?';
      continue;
    }
    Sha512 sh;
    sh.init(&s_buf[threadIdx.x], &s_h[threadIdx.x]);
    sh.put_str(kLoc0, sizeof(kLoc0) - 1);
    sh.put_u32_dec(start + r);
    sh.put_str(kLoc1, sizeof(kLoc1) - 1);
    sh.put_u32_dec(start);
    sh.put_str(kLoc2, sizeof(kLoc2) - 1);
    sh.put_str(seq_digest + size_t(c) * AVDB_DIGEST_CHARS, AVDB_DIGEST_CHARS);
    sh.put_str(kLoc3, sizeof(kLoc3) - 1);
    sh.finish();
    char loc[AVDB_DIGEST_CHARS];
    t24u(sh, loc);
    sh.init(&s_buf[threadIdx.x], &s_h[threadIdx.x]);
    sh.put_str(kAl0, sizeof(kAl0) - 1);
    sh.put_str(loc, AVDB_DIGEST_CHARS);
    sh.put_str(kAl1, sizeof(kAl1) - 1);
    sh.put_bytes(heap + off[i] + r, a);
    sh.put_str(kAl2, sizeof(kAl2) - 1);
    sh.finish();
    t24u(sh, o);
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

extern "C" int avdb_vrs_digest_workspace_size(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = 256 + 4 * n;
  return AVDB_OK;
}

extern "C" int avdb_vrs_digest(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                               const uint64_t* allele_off, const uint32_t* ref_len,
                               const uint32_t* alt_len, const uint8_t* heap, size_t n,
                               uint32_t max_seq_len, void* workspace, size_t workspace_bytes,
                               char* digest_out, uint8_t* is_long, void* stream) {
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  if (n == 0) return AVDB_OK;
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap || !digest_out) {
    avdb_set_error("avdb_vrs_digest: null array");
    return AVDB_EINVAL;
  }
  if (!ctx->has_digests || !ctx->d_seq_digest) {
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
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* count = static_cast<unsigned int*>(workspace);
  auto* list = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + 256);
  AVDB_HIP_TRY(hipMemsetAsync(count, 0, sizeof(unsigned int), s));
  const unsigned g1 = stream_grid(n, kBlock * 8, 4096);
  hipLaunchKernelGGL(k_long_compact, dim3(g1), dim3(kBlock), 0, s, ref_len, alt_len, n,
                     max_seq_len, is_long, list, count);
  AVDB_LAUNCH_CHECK("k_long_compact");
  // persistent grid over the compacted list: 4 workgroups per CU
  hipLaunchKernelGGL(k_vrs_digest, dim3(1024), dim3(kBlock), 0, s, chrom, pos, allele_off,
                     ref_len, alt_len, heap, list, count, ctx->d_seq_digest, ctx->tab.n, digest_out);
  AVDB_LAUNCH_CHECK("k_vrs_digest");
  return AVDB_OK;
}
