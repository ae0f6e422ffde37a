/*
 * avdb_oracle.c — plain-C CPU restatement of the AnnotatedVDB bin/key path.
 * TEST INFRASTRUCTURE ONLY: linked by tests/ and bench.py's cpu_baseline leg,
 * never by the product library.  Same record layout as include/avdb.h.
 *
 * Each function cites the reference behaviour it restates (paths relative to
 * NIAGADS/AnnotatedVDB); parity of this restatement is pinned by the golden
 * vectors in tests/golden (tests/test_oracle_golden.py).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define BIN_NONE 0xFFFFFFFFu
#define LEAF 15625u

/* smallest enclosing BinIndexRef row: bin_index.py:59-75 (end defaults to
 * start :63) + generate_bin_index_references.py:46-83 ((lo,hi] rows, level l
 * width 64e6>>(l-1), clipped at the chromosome length). */
static uint32_t bin_one(uint32_t c, uint32_t s, uint32_t e, int nchrom, const uint32_t* len,
                        uint8_t* st) {
  if ((int)c >= nchrom) { *st = 1; return BIN_NONE; }
  uint8_t status = 0;
  uint32_t lo = s, hi = e;
  if (e < s) { lo = e; hi = s; status = 3; }
  if (lo < 1 || hi > len[c]) { *st = 2; return BIN_NONE; }
  uint32_t qs = (lo - 1) / LEAF, qe = (hi - 1) / LEAF, x = qs ^ qe;
  int blen = 0;
  while (x) { ++blen; x >>= 1; }
  int level = blen <= 12 ? 13 - blen : 0;
  uint32_t idx = level ? qs >> (13 - level) : 0;
  *st = status;
  return ((uint32_t)level << 28) | idx;
}

void avdb_oracle_bin_assign(const uint8_t* chrom, const uint32_t* start, const uint32_t* end,
                            size_t n, const uint32_t* len, int nchrom, uint32_t* code,
                            uint8_t* status) {
  for (size_t i = 0; i < n; ++i) {
    uint8_t st;
    code[i] = bin_one(chrom[i], start[i], end ? end[i] : start[i], nchrom, len, &st);
    if (status) status[i] = st;
  }
}

/* end inference: variant_annotator.py:36-79, lcp from __normalize_alleles :82-121 */
static uint32_t end_one(const uint8_t* heap, uint64_t off, uint32_t r, uint32_t a, uint32_t pos,
                        uint32_t* lcp) {
  if (r == 1 && a == 1) { *lcp = 0; return pos; }
  const uint8_t* ref = heap + off;
  const uint8_t* alt = ref + r;
  uint32_t m = r < a ? r : a, k = 0;
  while (k < m && ref[k] == alt[k]) ++k;
  *lcp = k;
  uint32_t nr = r - k, na = a - k;
  if (r == a) {
    int inv = 1;
    for (uint32_t i = 0; i < r; ++i)
      if (ref[i] != alt[r - 1 - i]) { inv = 0; break; }
    return inv ? pos + r - 1 : pos + nr - 1;
  }
  if (na >= 1) return nr >= 1 ? pos + nr : (r > 1 ? pos + r - 1 : pos + 1);
  return nr == 0 ? pos + r - 1 : pos + nr;
}

void avdb_oracle_record_prep(const uint8_t* chrom, const uint32_t* pos, const uint64_t* off,
                             const uint32_t* rl, const uint32_t* al, const uint8_t* heap, size_t n,
                             const uint32_t* len, int nchrom, uint32_t* end, uint32_t* code,
                             uint8_t* status, uint32_t* lcp) {
  for (size_t i = 0; i < n; ++i) {
    uint32_t l;
    uint32_t e = end_one(heap, off[i], rl[i], al[i], pos[i], &l);
    uint8_t st;
    end[i] = e;
    code[i] = bin_one(chrom[i], pos[i], e, nchrom, len, &st);
    status[i] = st;
    if (lcp) lcp[i] = l;
  }
}

/* keep-first-occurrence dedup over primary keys (primary_key_generator.py:99-122;
 * removeDuplicates.sql:2-24).  Grouped form: equal (chrom,pos) are contiguous. */
static int same(const uint8_t* heap, const uint64_t* off, const uint32_t* rl, const uint32_t* al,
                const uint64_t* ext, size_t i, size_t j) {
  if (rl[i] != rl[j] || al[i] != al[j]) return 0;
  if (ext && ext[i] != ext[j]) return 0;
  return memcmp(heap + off[i], heap + off[j], (size_t)rl[i] + al[i]) == 0;
}

uint64_t avdb_oracle_dedup_grouped(const uint8_t* chrom, const uint32_t* pos, const uint64_t* off,
                                   const uint32_t* rl, const uint32_t* al, const uint8_t* heap,
                                   const uint64_t* ext, size_t n, uint8_t* keep) {
  uint64_t dups = 0;
  size_t run = 0;
  for (size_t i = 0; i < n; ++i) {
    if (i == 0 || chrom[i] != chrom[i - 1] || pos[i] != pos[i - 1]) run = i;
    uint8_t k = 1;
    for (size_t j = run; j < i; ++j)
      if (same(heap, off, rl, al, ext, i, j)) { k = 0; break; }
    keep[i] = k;
    dups += !k;
  }
  return dups;
}

/* ---- SHA-512 (FIPS 180-4) for sha512t24u checks ---- */
static const uint64_t K[80] = {
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

#define ROR(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

static void block(uint64_t* h, const uint8_t* p) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) {
    w[t] = 0;
    for (int b = 0; b < 8; ++b) w[t] = (w[t] << 8) | p[8 * t + b];
  }
  for (int t = 16; t < 80; ++t) {
    uint64_t s0 = ROR(w[t - 15], 1) ^ ROR(w[t - 15], 8) ^ (w[t - 15] >> 7);
    uint64_t s1 = ROR(w[t - 2], 19) ^ ROR(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 80; ++t) {
    uint64_t t1 = hh + (ROR(e, 14) ^ ROR(e, 18) ^ ROR(e, 41)) + ((e & f) ^ (~e & g)) + K[t] + w[t];
    uint64_t t2 = (ROR(a, 28) ^ ROR(a, 34) ^ ROR(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void avdb_oracle_sha512(const uint8_t* msg, size_t len, uint8_t out[64]) {
  uint64_t h[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                   0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                   0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
  size_t i = 0;
  for (; i + 128 <= len; i += 128) block(h, msg + i);
  uint8_t tail[256];
  size_t r = len - i;
  memset(tail, 0, sizeof(tail));
  memcpy(tail, msg + i, r);
  tail[r] = 0x80;
  size_t tl = (r + 1 + 16 <= 128) ? 128 : 256;
  uint64_t bits = (uint64_t)len * 8;
  for (int b = 0; b < 8; ++b) tail[tl - 1 - b] = (uint8_t)(bits >> (8 * b));
  block(h, tail);
  if (tl == 256) block(h, tail + 128);
  for (int k = 0; k < 8; ++k)
    for (int b = 0; b < 8; ++b) out[8 * k + b] = (uint8_t)(h[k] >> (56 - 8 * b));
}

/* ---- sha512t24u + VRS 1.x Allele digest (compute_vrs_identifier,
 * primary_key_generator.py:147-165; serialisation as oracle/avdb_oracle.py
 * vrs_allele_digest — PARITY UNPINNED vs vrs-python) ---- */
static const char B64URL[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

static void t24u(const uint8_t* msg, size_t len, char out[32]) {
  uint8_t h[64];
  avdb_oracle_sha512(msg, len, h);
  for (int g = 0; g < 8; ++g) {
    uint32_t v = ((uint32_t)h[3 * g] << 16) | ((uint32_t)h[3 * g + 1] << 8) | h[3 * g + 2];
    for (int k = 0; k < 4; ++k) out[4 * g + k] = B64URL[(v >> (18 - 6 * k)) & 63];
  }
}

static size_t put_str(uint8_t* o, const char* s) {
  size_t n = strlen(s);
  memcpy(o, s, n);
  return n;
}

static size_t put_u32(uint8_t* o, uint32_t v) {
  char t[16];
  int k = 0;
  do { t[k++] = (char)('0' + v % 10); v /= 10; } while (v);
  for (int i = 0; i < k; ++i) o[i] = (uint8_t)t[k - 1 - i];
  return (size_t)k;
}

/* digest_out[i*32..] for every record with rl+al > max_len (others untouched);
 * seq_digest: 32 chars per contig.  buf: scratch of >= 256 + max alt bytes. */
void avdb_oracle_vrs_digest(const uint8_t* chrom, const uint32_t* pos, const uint64_t* off,
                            const uint32_t* rl, const uint32_t* al, const uint8_t* heap, size_t n,
                            uint32_t max_len, const char* seq_digest, int nchrom, uint8_t* buf,
                            char* digest_out) {
  for (size_t i = 0; i < n; ++i) {
    if ((uint64_t)rl[i] + al[i] <= max_len) continue;
    if ((int)chrom[i] >= nchrom) { memset(digest_out + 32 * i, '?', 32); continue; }
    const uint32_t s = pos[i] - 1, e = s + rl[i];
    size_t k = 0;
    k += put_str(buf + k, "{\"interval\":{\"end\":{\"type\":\"Number\",\"value\":");
    k += put_u32(buf + k, e);
    k += put_str(buf + k, "},\"start\":{\"type\":\"Number\",\"value\":");
    k += put_u32(buf + k, s);
    k += put_str(buf + k, "},\"type\":\"SequenceInterval\"},\"sequence_id\":\"");
    memcpy(buf + k, seq_digest + 32 * chrom[i], 32);
    k += 32;
    k += put_str(buf + k, "\",\"type\":\"SequenceLocation\"}");
    char loc[32];
    t24u(buf, k, loc);
    k = put_str(buf, "{\"location\":\"");
    memcpy(buf + k, loc, 32);
    k += 32;
    k += put_str(buf + k, "\",\"state\":{\"sequence\":\"");
    memcpy(buf + k, heap + off[i] + rl[i], al[i]);
    k += al[i];
    k += put_str(buf + k, "\",\"type\":\"LiteralSequenceExpression\"},\"type\":\"Allele\"}");
    t24u(buf, k, digest_out + 32 * i);
  }
}

/* primary keys (primary_key_generator.py:99-122): label:pos:ref:alt[:rs<ext>],
 * or label:pos:<digest>[:rs<ext>] when rl+al > max_len; labels chr1..22,X,Y,M
 * -> "1".."22","X","Y","M" (enums/chromosomes.py:9-38).  Keys concatenated in
 * out, out_off[n+1]; returns the bytes written. */
static const char* LABEL[25] = {"1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12", "13",
                                "14", "15", "16", "17", "18", "19", "20", "21", "22", "X", "Y", "M"};

size_t avdb_oracle_primary_keys(const uint8_t* chrom, const uint32_t* pos, const uint64_t* off,
                                const uint32_t* rl, const uint32_t* al, const uint8_t* heap,
                                const uint64_t* ext, const char* digest, size_t n, uint32_t max_len,
                                uint8_t* out, uint64_t* out_off) {
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    out_off[i] = k;
    k += put_str(out + k, LABEL[chrom[i] < 25 ? chrom[i] : 0]);
    out[k++] = ':';
    k += put_u32(out + k, pos[i]);
    out[k++] = ':';
    if ((uint64_t)rl[i] + al[i] > max_len) {
      memcpy(out + k, digest + 32 * i, 32);
      k += 32;
    } else {
      memcpy(out + k, heap + off[i], rl[i]);
      k += rl[i];
      out[k++] = ':';
      memcpy(out + k, heap + off[i] + rl[i], al[i]);
      k += al[i];
    }
    if (ext && ext[i]) {
      char t[24];
      int d = 0;
      uint64_t v = ext[i];
      do { t[d++] = (char)('0' + v % 10); v /= 10; } while (v);
      k += put_str(out + k, ":rs");
      for (int q = 0; q < d; ++q) out[k++] = (uint8_t)t[d - 1 - q];
    }
  }
  out_off[n] = k;
  return k;
}

/* ltree bin paths (generate_bin_index_references.py:54,60-61,74): "chr<label>"
 * then ".L<l>.B<k>" for l = 1..level, k = global index at level 1 + 1, else the
 * index's lowest bit + 1 (B restarts under every parent).  BIN_NONE -> empty
 * text (K7's convention for an unmappable record).  Concatenated in out,
 * out_off[n+1]; returns the bytes written. */
size_t avdb_oracle_bin_paths(const uint8_t* chrom, const uint32_t* code, size_t n, uint8_t* out,
                             uint64_t* out_off) {
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    out_off[i] = k;
    if (code[i] == BIN_NONE || chrom[i] >= 25) continue;
    const uint32_t level = code[i] >> 28, g = code[i] & 0x0FFFFFFFu;
    k += put_str(out + k, "chr");
    k += put_str(out + k, LABEL[chrom[i]]);
    for (uint32_t l = 1; l <= level; ++l) {
      const uint32_t gl = g >> (level - l);
      k += put_str(out + k, ".L");
      k += put_u32(out + k, l);
      k += put_str(out + k, ".B");
      k += put_u32(out + k, l == 1 ? gl + 1 : (gl & 1) + 1);
    }
  }
  out_off[n] = k;
  return k;
}
