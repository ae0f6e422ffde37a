/*
 * cpu_baseline.c — SURVEY.md §8d(2): the "C -O3 OpenMP closed-form baseline on all
 * host cores, as a stronger comparator" beside the reference-structured Python
 * port.  TEST / BENCH INFRASTRUCTURE ONLY: loaded by bench.py's cpu_baseline leg,
 * never by the product library.  It runs the C oracle's own per-record functions
 * (avdb_oracle.c, included below: the restatement the parity tests pin) over the
 * batch with OpenMP — one closed form per record instead of the reference's
 * per-call Python and its one-bin cache — so it is the fastest CPU form of the same
 * arithmetic this repository has, not the reference's CPU path.
 */
#include "avdb_oracle.c"

#include <omp.h>
#include <stdlib.h>

/* BinIndex.find_bin_index (bin_index.py:59-75) for every record, closed form;
 * static schedule over `threads` threads. */
void avdb_cpubase_bin_assign(const uint8_t* chrom, const uint32_t* start, const uint32_t* end, size_t n,
                             const uint32_t* len, int nchrom, uint32_t* code, uint8_t* status, int threads) {
  const long long nn = (long long)n;
#pragma omp parallel for schedule(static) num_threads(threads)
  for (long long i = 0; i < nn; ++i) {
    uint8_t st;
    code[i] = bin_one(chrom[i], start[i], end ? end[i] : start[i], nchrom, len, &st);
    status[i] = st;
  }
}

/* The keyed record path (the C4k / C5 step: end inference + bin, VRS digests of
 * the long records, primary keys, ltree paths, keep-first dedup) over chunks of
 * `chunk` records, dynamically scheduled over `threads` threads.  end / code /
 * status / keep / digest are written for every record; the key and path text of a
 * chunk is rendered into that thread's scratch (its bytes are counted, not kept).
 * A run of equal (chrom, pos) cut by a chunk boundary is deduplicated per side (at
 * dbSNP density a handful of records per chunk).  Returns the text bytes. */
uint64_t avdb_cpubase_keyed(const uint8_t* chrom, const uint32_t* pos, const uint64_t* off, const uint32_t* rl,
                            const uint32_t* al, const uint8_t* heap, const uint64_t* ext, size_t n,
                            const uint32_t* len, int nchrom, uint32_t max_len, const char* seq_digest,
                            uint32_t* end, uint32_t* code, uint8_t* status, uint8_t* keep, char* digest,
                            size_t chunk, size_t max_allele_bytes, int threads) {
  uint64_t total = 0;
  const long long nc = (long long)((n + chunk - 1) / chunk);
#pragma omp parallel num_threads(threads) reduction(+ : total)
  {
    uint8_t* keys = (uint8_t*)malloc(chunk * 69 + chunk * (max_allele_bytes + 8) + 8);
    uint8_t* paths = (uint8_t*)malloc(chunk * 98 + 8);
    uint64_t* koff = (uint64_t*)malloc((chunk + 1) * sizeof(uint64_t));
    uint64_t* poff = (uint64_t*)malloc((chunk + 1) * sizeof(uint64_t));
    uint8_t* buf = (uint8_t*)malloc(256 + max_allele_bytes);
#pragma omp for schedule(dynamic, 1)
    for (long long c = 0; c < nc; ++c) {
      const size_t a = (size_t)c * chunk, m = (a + chunk <= n ? chunk : n - a);
      avdb_oracle_record_prep(chrom + a, pos + a, off + a, rl + a, al + a, heap, m, len, nchrom, end + a, code + a,
                              status + a, NULL);
      avdb_oracle_vrs_digest(chrom + a, pos + a, off + a, rl + a, al + a, heap, m, max_len, seq_digest, nchrom, buf,
                             digest + 32 * a);
      total += avdb_oracle_primary_keys(chrom + a, pos + a, off + a, rl + a, al + a, heap, ext + a, digest + 32 * a,
                                        m, max_len, keys, koff);
      total += avdb_oracle_bin_paths(chrom + a, code + a, m, paths, poff);
      avdb_oracle_dedup_grouped(chrom + a, pos + a, off + a, rl + a, al + a, heap, ext + a, m, keep + a);
    }
    free(keys);
    free(paths);
    free(koff);
    free(poff);
    free(buf);
  }
  return total;
}
