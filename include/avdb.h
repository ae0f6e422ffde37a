/*
 * avdb.h — C ABI of libavdb_hip.so, the MI355X (gfx950) kernel library behind
 * the AnnotatedVDB batch variant -> genomic-bin / primary-key path.
 *
 * Plain C: no torch or HIP types in any signature.  Every entry point returns
 * an int status (AVDB_OK == 0; negative on failure, message via
 * avdb_last_error()).  Array arguments are DEVICE pointers (HBM) unless marked
 * "host"; the caller owns every buffer.  `stream` is a hipStream_t passed as
 * void* (NULL = the device's null stream); all device work is enqueued on it
 * and nothing synchronises, so callers may capture the calls into a hipGraph.
 *
 * Reference interfaces replaced (paths relative to NIAGADS/AnnotatedVDB):
 *   - BinIndex.find_bin_index(chrm, start, end=None)      BinIndex/lib/python/bin_index.py:59-75
 *     and the external SQL find_bin_index(chr,start,end) it calls through
 *     BIN_INDEX_SQL (bin_index.py:9-14, _update_current_bin_index :43-56)
 *   - the BinIndexRef table it searches        BinIndex/bin/generate_bin_index_references.py:46-83
 *   - VariantAnnotator.infer_variant_end_location  Util/lib/python/variant_annotator.py:36-79
 *     and __normalize_alleles (common-prefix trim)  variant_annotator.py:82-121
 *   - VariantPKGenerator.generate_primary_key / compute_vrs_identifier
 *                                               Util/lib/python/primary_key_generator.py:99-165
 *   - the per-alt record-prep loop              Util/lib/python/loaders/vcf_variant_loader.py:259-348
 *   - in-batch duplicate-key semantics          Load/lib/sql/annotatedvdb_schema/patches/removeDuplicates.sql:2-24
 *
 * Record layout (structure of arrays, one entry per alt allele):
 *   chrom      u8[n]   contig code, index into the context's chromosome table
 *                      (default order chr1..chr22, chrX, chrY, chrM —
 *                      Util/lib/python/enums/chromosomes.py:9-38)
 *   pos/start  u32[n]  1-based VCF POS
 *   end        u32[n]  1-based inclusive end (nullable => end = start, bin_index.py:63)
 *   allele_off u64[n]  byte offset of the REF allele in `heap`; ALT follows at
 *                      allele_off + ref_len (raw, un-normalised VCF bytes)
 *   ref_len    u32[n], alt_len u32[n]
 *   ext_id     u64[n]  external id key (refSNP); 0 = none; equal keys <=> equal ids
 *   heap_bytes         size of the heap allocation: kernels read allele bytes as
 *                      8-byte-aligned words and never touch memory outside
 *                      [heap, heap + heap_bytes)
 *
 * Bin code (u32): level in bits 31..28 (0 = whole chromosome .. 13 = 15,625 bp
 * leaf), 0-based index of the bin at that level in bits 27..0.  The ltree path
 * "chrN.L1.B<k>...L<level>.B<k>" is a pure function of (chrom, code):
 * avdb_format_bin_path().  AVDB_BIN_NONE marks an unmappable record (the
 * reference raises TypeError there, bin_index.py:75).
 */
#ifndef AVDB_H_
#define AVDB_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: avdb_format_opts gained struct_size (first field) and adsp_dup; K5h/K8h/K1h
 *    host entries; AVDB_KEY_OVERFLOW / AVDB_PATH_OVERFLOW key states */
#define AVDB_ABI_VERSION 2

/* return codes */
#define AVDB_OK 0
#define AVDB_EINVAL (-1)   /* bad argument (null ctx, n too large, misaligned ...) */
#define AVDB_EHIP (-2)     /* HIP runtime error (launch / allocation) */
#define AVDB_ENOMEM (-3)
#define AVDB_ERANGE (-4)   /* output buffer too small */
#define AVDB_ERCCL (-5)    /* RCCL could not be loaded, or a collective failed */

/* per-record status (u8) */
#define AVDB_STATUS_OK 0
#define AVDB_STATUS_UNKNOWN_CHROM 1
#define AVDB_STATUS_OUT_OF_RANGE 2      /* start < 1 or end > chromosome length */
#define AVDB_STATUS_END_BEFORE_START 3  /* bin of [end,start]; reference answer is cache-history dependent */

#define AVDB_BIN_NONE 0xFFFFFFFFu
#define AVDB_N_LEVELS 14
#define AVDB_MAX_CHROM 64
#define AVDB_DIGEST_CHARS 32            /* sha512t24u: 24 bytes, base64url, no padding */
#define AVDB_MAX_PATH 128

/* counters[] slots (u64, accumulated) written by avdb_bin_assign / avdb_record_prep
 * (records, per-status) and avdb_pk_dedup / avdb_vrs_digest (dup/collision/long);
 * slots [0..15] are reserved */
#define AVDB_CTR_STATUS0 16             /* [16..19]: records per status */
#define AVDB_CTR_RECORDS 20
#define AVDB_CTR_DUPLICATES 21          /* records whose primary key repeats an earlier one */
#define AVDB_CTR_HASH_COLLISIONS 22     /* fingerprint collisions resolved by byte compare */
#define AVDB_CTR_LONG 23                /* records with ref_len + alt_len > max_seq_len */
#define AVDB_CTR_COPY_ROWS 24           /* COPY rows written by avdb_vcf_format_write */
#define AVDB_CTR_SKIPPED_ALTS 25        /* ALT '.' entries skipped (vcf_variant_loader.py:277-280) */
#define AVDB_CTR_DUP_ROWS 26            /* records whose COPY row was dropped (keep == 0) */
#define AVDB_CTR_HOST_LINES 27          /* lines left to the host renderer */
#define AVDB_CTR_EXISTING 28            /* records found in the existing-variant key set (K6) */
#define AVDB_CTR_ADSP_UPDATES 29        /* ADSP records whose key was already loaded (is_adsp_variant UPDATEs) */
#define AVDB_N_COUNTERS 32

typedef struct avdb_ctx avdb_ctx;

int avdb_abi_version(void);
/* Thread-local description of the last failure in this thread. */
const char* avdb_last_error(void);
int avdb_device_count(int* n);

/* ---- context -----------------------------------------------------------
 * One context per device.  chrom_len (host) gives each contig's length; it is
 * the information BinIndexRef carries (generate_bin_index_references.py:17-43).
 * Not thread-safe per context; calls are ordered on the caller's stream.  */
int avdb_ctx_create(int device, const uint32_t* chrom_len_host, int n_chrom, avdb_ctx** out);
int avdb_ctx_destroy(avdb_ctx* ctx);
/* Launch-shape options of a context (same results, another grid):
 *   AVDB_OPT_K4_GRID  workgroups of K4's persistent digest grid, 0 = its occupancy on
 *                     every CU (the default); fewer leave CUs to K7 running beside K4
 *                     on another stream (AVDB_KEYS_DIGEST_DEFERRED).
 */
#define AVDB_OPT_K4_GRID 1
/*   AVDB_OPT_K7_GRID  workgroups (one wave each) of K7's write pass, 0 = the default; a
 *                     persistent grid below the chip's occupancy leaves registers to K4 */
#define AVDB_OPT_K7_GRID 2
int avdb_ctx_set_option(avdb_ctx* ctx, int option, int64_t value);
int avdb_ctx_n_chrom(const avdb_ctx* ctx);
/* GA4GH refget digests (32 chars each, no "ga4gh:SQ." prefix) of every contig,
 * host array n_chrom*32 bytes; required only by avdb_vrs_digest. */
int avdb_ctx_set_sequence_digests(avdb_ctx* ctx, const char* digests_host, int n_chrom);
/* Number of L8 (500 kb) bins over the whole chromosome table (histogram size). */
int avdb_l8_bin_count(const avdb_ctx* ctx, uint32_t* n_bins);

/* ---- K1: smallest enclosing bin ----------------------------------------
 * Replaces BinIndex.find_bin_index + SQL find_bin_index (bin_index.py:43-75).
 * end may be NULL (end = start); status may be NULL.  If hist_l8 (u32[n_l8])
 * and/or counters (u64[AVDB_N_COUNTERS]) are non-NULL they are ACCUMULATED
 * (caller zeroes them): L8 bin of `start` for every mappable record, records
 * and records per status. */
int avdb_bin_assign(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* start,
                    const uint32_t* end, size_t n, uint32_t* bin_code, uint8_t* status,
                    uint32_t* hist_l8, uint64_t* counters, void* stream);

/* ---- K2: record prep (end inference + bin, fused) ------------------------
 * Per alt allele: common-prefix length of ref/alt (variant_annotator.py:82-121),
 * inferred end (variant_annotator.py:36-79), then the bin of [pos,end]
 * (vcf_variant_loader.py:310-311).  end_out/bin_code required; status, lcp,
 * hist_l8, counters optional (NULL).  */
int avdb_record_prep(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                     const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                     const uint8_t* heap, size_t heap_bytes, size_t n, uint32_t* end_out,
                     uint32_t* bin_code,
                     uint8_t* status, uint32_t* lcp, uint32_t* hist_l8, uint64_t* counters,
                     void* stream);

/* ---- K3: in-batch primary-key dedup --------------------------------------
 * keep[i] = 1 iff no j < i has the same primary key chr:pos:ref:alt[:ext]
 * (primary_key_generator.py:99-122; equal keys <=> equal (chrom,pos,ref,alt,ext_id)).
 * grouped != 0 promises records with equal (chrom,pos) are contiguous (any
 * position-sorted VCF): a run scan; a 16-byte-aligned `workspace` of at least
 * 16384 + 4*round_up(n, 4) bytes (optional) lets it list the records that share
 * their predecessor's position and resolve only those (faster).  grouped == 0: hash
 * path, needs `workspace` of avdb_pk_dedup_workspace_size() bytes (device).
 * counters[AVDB_CTR_DUPLICATES / _HASH_COLLISIONS] accumulated if non-NULL. */
int avdb_pk_dedup_workspace_size(size_t n, size_t* bytes);
int avdb_pk_dedup(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                  const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                  const uint8_t* heap, size_t heap_bytes, const uint64_t* ext_id, size_t n,
                  int grouped,
                  void* workspace, size_t workspace_bytes, uint8_t* keep, uint64_t* counters,
                  void* stream);
/* The same (grouped, list form) with flags: AVDB_DEDUP_MARKED = avdb_record_prep_keyed
 * already ran the first phase for this batch (keep = 1 everywhere, the records that
 * share their predecessor's position listed in `workspace`, which must be the one it
 * was given, with `keep` its keep array): only the run scan over those lists runs. */
#define AVDB_DEDUP_MARKED 1u
/* With AVDB_DEDUP_MARKED: the marks came from avdb_keyed_prep (its list layout). */
#define AVDB_DEDUP_ONEPASS 2u
int avdb_pk_dedup_ex(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                     const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                     const uint64_t* ext_id, size_t n, void* workspace, size_t workspace_bytes, uint8_t* keep,
                     uint64_t* counters, uint32_t flags, void* stream);

/* ---- K4: digests ---------------------------------------------------------
 * sha512t24u of n byte strings (data + off[i], len[i]) -> out[i*32..] base64url. */
int avdb_sha512t24u(avdb_ctx* ctx, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                    size_t n, char* out, void* stream);
/* Long-allele key digest (compute_vrs_identifier, primary_key_generator.py:147-165):
 * for every record with ref_len + alt_len > max_seq_len, the VRS-1.x Allele
 * digest of interval (pos-1, pos-1+ref_len] and literal state ALT, written to
 * digest_out[i*32..] (other rows untouched); is_long[i] set 0/1 if non-NULL.
 * Long rows are compacted into `workspace` (avdb_vrs_digest_workspace_size()
 * bytes, device, 16-byte aligned) first.  PARITY UNPINNED. */
int avdb_vrs_digest_workspace_size(size_t n, size_t* bytes);
int avdb_vrs_digest(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                    const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                    const uint8_t* heap, size_t heap_bytes, size_t n, uint32_t max_seq_len,
                    void* workspace,
                    size_t workspace_bytes, char* digest_out, uint8_t* is_long, void* stream);
/* The same with flags: AVDB_DIGEST_CODES_READY = avdb_record_prep_keyed already
 * classified this batch's records into the workspace (same n and max_seq_len), so
 * the pass over both length arrays is replaced by one over those bytes. */
#define AVDB_DIGEST_CODES_READY 1u
int avdb_vrs_digest_ex(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                       const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                       size_t n, uint32_t max_seq_len, void* workspace, size_t workspace_bytes, char* digest_out,
                       uint8_t* is_long, uint32_t flags, void* stream);
/* The same, and every long record's 32 characters also written into the key text
 * of a deferred K7 / avdb_keyed_prep call on the same batch (key_off / key_out /
 * key_state: that call's; the keys in state AVDB_KEY_DIGEST_PENDING get them at
 * key_off[i] + len("label:pos:") and become AVDB_KEY_OK) — the work of
 * avdb_primary_keys_fill_digests without its pass over every record. */
int avdb_vrs_digest_keys(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                         const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                         size_t n, uint32_t max_seq_len, void* workspace, size_t workspace_bytes, char* digest_out,
                         uint8_t* is_long, uint32_t flags, const uint64_t* key_off, uint8_t* key_out,
                         uint8_t* key_state, void* stream);

/* ---- K0: VCF text -> per-alt record SoA ----------------------------------
 * Replaces the text half of VcfEntryParser.parse_entry / get_variant / get_refsnp
 * (Util/lib/python/parsers/vcf_parser.py:76-169) and the per-alt loop head of
 * VCFVariantLoader.__parse_alt_alleles (vcf_variant_loader.py:273-280) for a batch
 * of VCF lines resident in device memory (`text`, '\n'-separated, as
 * load_vcf_file.py:101-119 reads them; each line is rstripped).
 *   1. avdb_vcf_count_lines  -> number of '\n' bytes (device u64); the caller derives
 *      n_lines = n_newlines + (text does not end in '\n').
 *   2. avdb_vcf_parse_lines  -> one avdb_vcf_line per line, plus exclusive prefix sums
 *      rec_off[n_lines+1] / heap_off[n_lines+1] of records and allele-heap bytes.
 *      `line_counts` is the workspace step 1 filled (its per-workgroup newline
 *      offsets are reused); NULL recounts.
 *   3. avdb_vcf_emit         -> the record SoA K2/K3/K4 consume (one row per ALT that
 *      is not '.', REF+ALT copied into `heap`), with rec_line/rec_alt back-references.
 * Text cases the GPU does not canonicalise are flagged for the host (flags below). */
#define AVDB_VCF_COMMENT 0x001u         /* starts with '#': not a data line */
#define AVDB_VCF_FEW_FIELDS 0x002u      /* < 8 tab-separated fields (IndexError, vcf_parser.py:98-100) */
#define AVDB_VCF_BAD_POS 0x004u         /* POS not a plain decimal < 2^32: host resolves */
#define AVDB_VCF_EXT_HOST 0x008u        /* refSNP id not canonical rs<N>: host interns ext_id */
#define AVDB_VCF_ID_RS 0x010u           /* 'rs' in ID: ref_snp_id = ID (vcf_parser.py:164) */
#define AVDB_VCF_INFO_RS 0x020u         /* ref_snp_id = 'rs' + INFO RS (vcf_parser.py:166-167) */
#define AVDB_VCF_ID_METASEQ 0x040u      /* ID is '.' or starts 'rs': variant id = chr:pos:ref:alt (:140-142) */
#define AVDB_VCF_CHROM_HOST 0x080u      /* CHROM has non-alphanumeric bytes: host resolves */
#define AVDB_VCF_EMPTY 0x100u           /* empty after rstrip */
#define AVDB_VCF_ID_HOST 0x200u         /* ID looks numeric (Python coerces it): host resolves */

typedef struct avdb_vcf_line {
  uint64_t start;         /* byte offset of the line in text */
  uint32_t len;           /* bytes after rstrip */
  uint32_t n_fields;      /* tab-separated fields */
  uint32_t field[8];      /* start of fields 0..7 relative to `start` (field k ends at field[k+1]-1) */
  uint32_t field_end8;    /* end of field 7 (INFO) relative to `start` */
  uint32_t pos;
  uint64_t ext_id;
  uint32_t n_alt;         /* ALT entries including '.' */
  uint32_t n_rec;         /* records emitted (ALT != '.') */
  uint32_t flags;
  uint8_t chrom;          /* contig code, 255 unknown */
  uint8_t pad[3];
} avdb_vcf_line;

#define AVDB_VCF_COUNT_WORKSPACE_BYTES 32768u /* minimum workspace of avdb_vcf_count_lines */
int avdb_vcf_workspace_size(size_t text_bytes, size_t n_lines, size_t* bytes);
/* Workspace of avdb_vcf_count_lines that also holds the newline count of every
 * parse window (AVDB_VCF_PARSE_WIN_KB pieces of the count pass's cut, 24 KB by
 * default): given that much, the count
 * pass writes them and avdb_vcf_parse_lines2 parses one window per workgroup,
 * finding the line starts itself, with no separate line-starts pass.  With only
 * AVDB_VCF_COUNT_WORKSPACE_BYTES the starts pass runs (same outputs). */
int avdb_vcf_count_workspace_size(size_t text_bytes, size_t* bytes);
int avdb_vcf_count_lines(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, void* workspace,
                         size_t workspace_bytes, uint64_t* n_newlines, void* stream);
/* Parse options (nullable = the default 8-field header, no chromosome map):
 *   min_fields  the loader's header width (VCFVariantLoader.set_vcf_header_fields,
 *               vcf_variant_loader.py:88-93,368, for a header whose first eight fields are
 *               the standard ones, e.g. a pVCF): a line with fewer values is flagged
 *               AVDB_VCF_FEW_FIELDS (the reference raises IndexError there);
 *   chrom_map   VcfEntryParser.update_chromosome (vcf_parser.py:117-124) with a
 *               ChromosomeMap (chromosome_map_parser.py:84-91): CHROM is looked up as
 *               bytes; a CHROM not in the map, or mapped to a key the host must
 *               resolve, is flagged AVDB_VCF_CHROM_HOST (the reference raises KeyError). */
typedef struct avdb_chrom_map avdb_chrom_map;
typedef struct avdb_vcf_opts {
  uint32_t struct_size;             /* sizeof(avdb_vcf_opts) */
  uint32_t min_fields;
  const avdb_chrom_map* chrom_map;  /* nullable */
} avdb_vcf_opts;
/* keys (host): the map's source ids, keys[key_off[k] .. key_off[k+1]); codes[k] (host):
 * the contig code of the chromosome source id k maps to, 0xFF = lines with this CHROM
 * are rendered by the caller.  The first of duplicate keys wins. */
int avdb_chrom_map_create(avdb_ctx* ctx, const uint8_t* keys_host, const uint64_t* key_off_host, size_t n_keys,
                          const uint8_t* codes_host, avdb_chrom_map** out);
int avdb_chrom_map_destroy(avdb_chrom_map* map);
int avdb_vcf_parse_lines(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                         const void* line_counts, void* workspace, size_t workspace_bytes,
                         avdb_vcf_line* lines,
                         uint64_t* rec_off, uint64_t* heap_off, const avdb_vcf_opts* opts, void* stream);
/* avdb_vcf_parse_lines with the size of `line_counts`: a count workspace of at
 * least avdb_vcf_count_workspace_size(text_bytes) bytes takes the window path. */
/* `lines` may be NULL here: no public line table is written (the tokenize-only
 * path), and what the emit needs of each line (32 bytes) goes into `workspace`
 * instead, for avdb_vcf_emit_ws with that same workspace. */
int avdb_vcf_parse_lines2(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                          const void* line_counts, size_t line_counts_bytes, void* workspace,
                          size_t workspace_bytes, avdb_vcf_line* lines, uint64_t* rec_off, uint64_t* heap_off,
                          const avdb_vcf_opts* opts, void* stream);
int avdb_vcf_emit(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                  const avdb_vcf_line* lines, const uint64_t* rec_off, const uint64_t* heap_off,
                  uint8_t* chrom, uint32_t* pos, uint64_t* allele_off, uint32_t* ref_len,
                  uint32_t* alt_len, uint64_t* ext_id, uint8_t* heap, uint32_t* rec_line,
                  uint32_t* rec_alt, void* stream);
/* avdb_vcf_emit after avdb_vcf_parse_lines2(..., lines = NULL, ...): the line data
 * comes from that call's workspace (same text_bytes and n_lines). */
int avdb_vcf_emit_ws(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                     const void* parse_workspace, size_t parse_workspace_bytes, const uint64_t* rec_off,
                     const uint64_t* heap_off, uint8_t* chrom, uint32_t* pos, uint64_t* allele_off,
                     uint32_t* ref_len, uint32_t* alt_len, uint64_t* ext_id, uint8_t* heap, uint32_t* rec_line,
                     uint32_t* rec_alt, void* stream);
/* The records without the count pass (the tokenize-only path, no line table):
 * avdb_vcf_parse_local parses one workgroup per parse window with no line numbers
 * known, each window writing its lines' counts, its records and their REF+ALT bytes
 * to slots of its own in `workspace` (avdb_vcf_local_workspace_size(text_bytes)
 * bytes, 16-byte aligned), from the text it has staged; one scan of the windows'
 * totals then gives every window its first line, record and heap byte.
 * totals (device, 4 x u64): lines, records, heap bytes, and the number of windows
 * the path could not take (more than AVDB_VCF_LOCAL_CAP = 1024 lines or records in
 * a 24 KB window, more than 24 KB of REF+ALT bytes in its records, or a line whose
 * records / heap bytes exceed 2^23).  With totals[3] == 0, avdb_vcf_emit_local moves
 * the slots into the same records, heap, rec_line / rec_alt and per-line rec_off /
 * heap_off (totals[0] + 1 entries each, nullable) as count -> parse ->
 * avdb_vcf_emit_ws write — coalesced copies; it does not read the text (`text` is
 * kept in the signature and may be NULL); with totals[3] != 0 the caller takes that
 * counted path.  The same workspace goes to both calls.  Workspace per 24 KB window
 * of text: 1,024 line slots of 8 bytes, 1,024 record slots of 32 bytes, 24 KB of
 * heap slots and 40 bytes of window totals, about 2.7x text_bytes at any size (a
 * one-line text: two windows, 128 KB); the slots are written only for the lines
 * and records present. */
int avdb_vcf_local_workspace_size(size_t text_bytes, size_t* bytes);
int avdb_vcf_parse_local(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, void* workspace,
                         size_t workspace_bytes, const avdb_vcf_opts* opts, uint64_t* totals, void* stream);
int avdb_vcf_emit_local(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, const void* workspace,
                        size_t workspace_bytes, uint64_t* rec_off, uint64_t* heap_off, uint8_t* chrom, uint32_t* pos,
                        uint64_t* allele_off, uint32_t* ref_len, uint32_t* alt_len, uint64_t* ext_id, uint8_t* heap,
                        uint32_t* rec_line, uint32_t* rec_alt, void* stream);

/* ---- K5: the load driver's text outputs ---------------------------------
 * Replaces the per-alt COPY row assembly of VCFVariantLoader.__parse_alt_alleles
 * (vcf_variant_loader.py:320-343) — primary key (primary_key_generator.py:99-122),
 * metaseq id, bin path, refSNP, multi-allelic flag, display attributes
 * (variant_annotator.py:134-241) and INFO FREQ allele frequencies
 * (vcf_parser.py:200-222), both as json.dumps text — and the .mapping line
 * (Load/bin/load_vcf_file.py:116-117), for lines K0 tokenized and K2 (end,
 * bin_code, status), K4 (digest, long keys; NULL if none) and K3 (keep; NULL =
 * keep all) processed.
 *   1. avdb_vcf_format_size : line_state[n_lines] and exclusive byte offsets
 *      copy_off[n_lines+1] / map_off[n_lines+1] (totals in [n_lines]);
 *      workspace of avdb_format_workspace_size(n_lines) bytes.
 *   2. avdb_vcf_format_write: the texts into copy_out / map_out (8-byte aligned,
 *      sized by the totals); counters[AVDB_CTR_COPY_ROWS..HOST_LINES] accumulated.
 * line_state: AVDB_LINE_GPU rendered here; AVDB_LINE_HOST zero bytes — the host
 * renders the line (text the GPU does not canonicalise, or a line on which the
 * reference raises); AVDB_LINE_SKIP comment line ('#', load_vcf_file.py:103). */
#define AVDB_LINE_GPU 0
#define AVDB_LINE_HOST 1
#define AVDB_LINE_SKIP 2
#define AVDB_MAX_ALG_ID 64

#define AVDB_FORMAT_ADSP 1u           /* opts.flags: COPY rows end with is_adsp_variant = True
                                        * (vcf_variant_loader.py:336-337) */
typedef struct avdb_format_opts {
  uint32_t struct_size;   /* sizeof(avdb_format_opts) as the caller compiled it: the
                           * library refuses a size it does not know (ABI check) */
  uint32_t max_seq_len;   /* primary_key_generator.py:53 (default 50) */
  const char* alg_id;     /* xstr(row_algorithm_id), host NUL-terminated; NULL = "" */
  uint32_t flags;         /* AVDB_FORMAT_* */
  /* --skipExisting (optional, device; NULL = off): K6 match / kind per record and
   * the .mapping text each existing key contributes (its match list, rendered
   * once by the host): frag[frag_off[k] .. frag_off[k+1]).  A matched record gets
   * no COPY row, its fragment in the .mapping line, and counts as skipped
   * (vcf_variant_loader.py:285-291). */
  const int32_t* match;
  const uint8_t* match_kind;
  const uint8_t* frag;
  const uint64_t* frag_off;
  /* ADSP datasource (optional, device; NULL = off): per record, nonzero when its
   * primary key is already loaded (K6 avdb_keyset_probe_text over K7's keys):
   * is_duplicate(recordPK) -> an is_adsp_variant UPDATE instead of a COPY row, no
   * .mapping entry, counters[AVDB_CTR_ADSP_UPDATES] (vcf_variant_loader.py:303-307). */
  const uint8_t* adsp_dup;
} avdb_format_opts;

int avdb_format_workspace_size(size_t n, size_t* bytes);
int avdb_vcf_format_size(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                         const avdb_vcf_line* lines, const uint64_t* rec_off, const uint32_t* end,
                         const uint32_t* bin_code, const uint8_t* status, const char* digest,
                         const uint8_t* keep, const avdb_format_opts* opts, void* workspace,
                         size_t workspace_bytes, uint64_t* copy_off, uint64_t* map_off,
                         uint8_t* line_state, void* stream);
int avdb_vcf_format_write(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                          const avdb_vcf_line* lines, const uint64_t* rec_off, const uint32_t* end,
                          const uint32_t* bin_code, const uint8_t* status, const char* digest,
                          const uint8_t* keep, const avdb_format_opts* opts, const uint64_t* copy_off,
                          const uint64_t* map_off, const uint8_t* line_state, uint8_t* copy_out,
                          uint8_t* map_out, uint64_t* counters, void* stream);
/* K5h: ONE line of VCF text (host memory, no newline needed) -> its COPY rows and
 * .mapping line, rendered by the library's host code with the kernels' own
 * per-line definitions (K0 parse_line, K2 infer_end/classify, K5 format_line).
 * The per-line call of the reference's loader (VCFVariantLoader.parse_variant,
 * vcf_variant_loader.py:351-391, called per line by load_vcf_file.py:112) pays no
 * GPU launch + sync this way.  res->state: AVDB_LINE_GPU = rendered (the same
 * bytes the K5 kernels write for this line), AVDB_LINE_HOST = the caller renders
 * it (same rules as K5: non-canonical text, long alleles, unmappable records, ...),
 * AVDB_LINE_SKIP = comment.  opts: alg_id, max_seq_len, flags (AVDB_FORMAT_ADSP);
 * vcf_opts (nullable): header width and chromosome map as for avdb_vcf_parse_lines;
 * match / adsp_dup must be NULL (batch features).  Returns AVDB_ERANGE when a
 * buffer is short (res holds the sizes).  A context made with device = -1
 * suffices; thread-safe per calling thread. */
typedef struct avdb_line_result {
  uint32_t state;
  uint32_t flags;        /* K0 AVDB_VCF_* flags of the line */
  uint32_t copy_bytes;   /* COPY rows written (each ends with '\n') */
  uint32_t map_bytes;    /* .mapping line written: id '\t' [ {...}, ... ] '\n' */
  uint32_t n_rec;        /* records (ALT != '.') */
  uint32_t n_rows;       /* COPY rows */
  uint32_t n_skip;       /* ALT '.' skipped */
  uint32_t n_dup;
  uint32_t n_upd;
  uint32_t reserved;
} avdb_line_result;
int avdb_vcf_line_host(const avdb_ctx* ctx, const char* line, size_t len, const avdb_format_opts* opts,
                       const avdb_vcf_opts* vcf_opts, char* copy_out, size_t copy_cap, char* map_out,
                       size_t map_cap, avdb_line_result* res);
/* get_display_attributes (variant_annotator.py:134-241) of a record batch as
 * json.dumps text (ASCII alleles; json escaping applied).  end = K2's end.
 * Call with out == NULL first: rec_state[i] (0 ok, 1 non-ASCII allele, 2 heap
 * overrun) and exclusive offsets out_off[n+1]; then with out (8-byte aligned,
 * out_off[n] bytes).  Contigs >= 25 get no label inside normalized_metaseq_id. */
int avdb_display_attributes(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint32_t* end,
                            const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                            const uint8_t* heap, size_t heap_bytes, size_t n, void* workspace,
                            size_t workspace_bytes, uint64_t* out_off, uint8_t* out, uint8_t* rec_state,
                            void* stream);

/* ---- K7: primary keys and bin paths of a record batch as text -----------
 * Replaces VariantPKGenerator.generate_primary_key (primary_key_generator.py:99-122,
 * the record_primary_key column) and the ltree text BinIndex.find_bin_index
 * returns (bin_index.py:75) for a whole record batch:
 *   key  = <contig label> ':' pos ':' ref ':' alt [':' 'rs'<ext_id>]   (short)
 *          <contig label> ':' pos ':' <digest>   [':' 'rs'<ext_id>]   (ref_len + alt_len
 *          > max_seq_len; digest = avdb_vrs_digest output, 32 chars per record)
 *   path = avdb_format_bin_path(chrom, bin_code) (bin_code NULL: no paths)
 * ext_id is rendered 'rs' + decimal (canonical refSNP keys, < 2^63).
 * Call with key_out == NULL first: exclusive offsets key_off[n+1] (and
 * path_off[n+1]) from the SoA alone; then with key_out (and path_out), 8-byte
 * aligned, of key_cap (path_cap) bytes >= the totals, which writes the text and
 * key_state[n] (a text that would end past its cap is not written, and its record's
 * state says so: AVDB_KEY_OVERFLOW / AVDB_PATH_OVERFLOW).  The write call runs the
 * one-pass write pass below (workspace: avdb_format_workspace_size(n) bytes, 16-byte
 * aligned) and writes the same key_off / path_off again: */
#define AVDB_KEY_OK 0
#define AVDB_KEY_HOST 1          /* ':' in an allele (the reference raises ValueError),
                                  * non-ASCII bytes, a contig without label or an
                                  * interned (non-rs) external id: caller renders */
#define AVDB_KEY_NEED_DIGEST 2   /* long record and digest == NULL */
#define AVDB_KEY_OVERFLOW 3      /* the key would end past key_cap: not written */
#define AVDB_KEY_DIGEST_PENDING 4 /* long record under AVDB_KEYS_DIGEST_DEFERRED: the key is
                                  * written except its 32 digest characters (zero bytes)
                                  * until avdb_primary_keys_fill_digests sets them and the
                                  * state to AVDB_KEY_OK */
#define AVDB_PATH_OVERFLOW 0x10u /* ORed in: the path would end past path_cap: not written */
int avdb_primary_keys(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                      const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap,
                      size_t heap_bytes, const uint64_t* ext_id, const uint32_t* bin_code,
                      const char* digest, size_t n, uint32_t max_seq_len, void* workspace,
                      size_t workspace_bytes, uint64_t* key_off, uint64_t* path_off, uint8_t* key_out,
                      size_t key_cap, uint8_t* path_out, size_t path_cap, uint8_t* key_state,
                      void* stream);

/* K7 without a host round trip: per group of 64 / 256 records the key and path
 * byte totals (or the keyed K2's), one scan over the group totals, then the write
 * pass, which recomputes each record's sizes from the SoA it reads anyway, writes
 * the offsets and renders the text.  Same inputs and outputs as
 * avdb_primary_keys, except that key_off[n+1] / path_off[n+1] are OUTPUTS and the
 * text buffers are sized in advance: avdb_primary_keys_bound gives capacities no
 * batch of n records with heap_bytes of alleles can exceed.  workspace:
 * avdb_primary_keys_onepass_workspace_size(n) bytes, 8-byte aligned. */
int avdb_primary_keys_bound(size_t n, size_t heap_bytes, size_t* key_cap, size_t* path_cap);
int avdb_primary_keys_onepass_workspace_size(size_t n, size_t* bytes);
int avdb_primary_keys_onepass(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                              const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap,
                              size_t heap_bytes, const uint64_t* ext_id, const uint32_t* bin_code,
                              const char* digest, size_t n, uint32_t max_seq_len, void* workspace,
                              size_t workspace_bytes, uint64_t* key_off, uint64_t* path_off, uint8_t* key_out,
                              size_t key_cap, uint8_t* path_out, size_t path_cap, uint8_t* key_state,
                              void* stream);
/* The same with flags: AVDB_KEYS_TOTALS_READY = the workspace already holds the
 * group totals avdb_record_prep_keyed wrote for this batch (same n, max_seq_len,
 * digest presence and paths), so the totals pass over the SoA is skipped (only
 * the last group is summed again, inside the scan). */
#define AVDB_KEYS_TOTALS_READY 1u
/* AVDB_KEYS_DIGEST_DEFERRED (digest == NULL): long records' keys are laid out with
 * their 32 digest characters still to come (state AVDB_KEY_DIGEST_PENDING), so K7
 * need not wait for K4: run avdb_vrs_digest beside it (another stream) and then
 * avdb_primary_keys_fill_digests.  The keyed K2 totals for this are the ones made
 * with has_digest != 0. */
#define AVDB_KEYS_DIGEST_DEFERRED 2u
/* AVDB_KEYS_OFF32: key_off / path_off in the narrow layout, each a buffer of
 * avdb_keys_off32_bytes(n) bytes (8-byte aligned): n + 1 uint32 low words (offset mod
 * 2^32), then from the next 8-byte boundary one uint64 base per 4,096 records (the
 * full offset of record 4096 k).  Full offset of i = base[i >> 12] +
 * (uint32_t)(low[i] - (uint32_t)base[i >> 12]) (4,096 records' text is < 4 GB).
 * 4 bytes per record and stream are written instead of 8.  Not accepted by
 * avdb_primary_keys_fill_digests / avdb_vrs_digest_keys / avdb_keyset_probe_text,
 * which take uint64 offsets. */
#define AVDB_KEYS_OFF32 4u
int avdb_keys_off32_bytes(size_t n, size_t* bytes);
int avdb_primary_keys_onepass_ex(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                 const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                                 const uint8_t* heap, size_t heap_bytes, const uint64_t* ext_id,
                                 const uint32_t* bin_code, const char* digest, size_t n, uint32_t max_seq_len,
                                 void* workspace, size_t workspace_bytes, uint64_t* key_off, uint64_t* path_off,
                                 uint8_t* key_out, size_t key_cap, uint8_t* path_out, size_t path_cap,
                                 uint8_t* key_state, uint32_t flags, void* stream);
/* The digest characters of every AVDB_KEY_DIGEST_PENDING key: digest = the
 * avdb_vrs_digest output for the same batch (32 chars per record, 16-byte
 * aligned), key_off / key_out / key_state = the deferred K7 call's (key_state
 * 16-byte aligned).  Each pending key's state becomes AVDB_KEY_OK. */
int avdb_primary_keys_fill_digests(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, size_t n,
                                   const char* digest, const uint64_t* key_off, uint8_t* key_out,
                                   uint8_t* key_state, void* stream);
/* K2 that also writes K7's group totals (key / path bytes per group of 64 or 256
 * records) into a one-pass K7 workspace, from the SoA it reads anyway plus the
 * refSNP ids: the record-prep half of the keyed pipeline (C4k, C1).  With a K4
 * workspace (avdb_vrs_digest_workspace_size(n) bytes, 16-byte aligned; nullable)
 * it also classifies every record for K4 (short, or long and its SHA-512 block
 * bucket).  With a K3 list workspace and a keep array (nullable) it also runs K3's
 * first phase (keep = 1; listed per workgroup: the records that share (chrom, pos)
 * with their predecessor and either have its ref / alt lengths and ext_id or are
 * third or later at their position — the others cannot repeat an earlier primary
 * key) when its lists fit (kDedupListHead + 4 * grid * slice bytes: at most
 * 16 KB + 4 (n + 2^22) at the default unroll).  The resolve (avdb_pk_dedup_ex with
 * AVDB_DEDUP_MARKED) must then be given the same ext_id.  key_workspace NULL: no
 * K7 totals (a step without key text, as C5's: K4's codes and K3's marks only).
 * *totals_written = AVDB_KEYED_TOTALS | AVDB_KEYED_LONG_CODES | AVDB_KEYED_DEDUP_MARKS
 * for what it wrote (16-byte aligned arrays; else 0 and it is avdb_record_prep):
 * pass AVDB_KEYS_TOTALS_READY to avdb_primary_keys_onepass_ex, AVDB_DIGEST_CODES_READY
 * to avdb_vrs_digest_ex (same n and max_seq_len) and AVDB_DEDUP_MARKED to
 * avdb_pk_dedup_ex then. */
#define AVDB_KEYED_TOTALS 1
#define AVDB_KEYED_LONG_CODES 2
#define AVDB_KEYED_DEDUP_MARKS 4
int avdb_record_prep_keyed(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                           const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                           size_t n, uint32_t* end_out, uint32_t* bin_code, uint8_t* status, uint32_t* lcp,
                           uint32_t* hist_l8, uint64_t* counters, const uint64_t* ext_id, uint32_t max_seq_len,
                           int has_digest, int with_paths, void* key_workspace, size_t key_workspace_bytes,
                           void* digest_workspace, size_t digest_workspace_bytes, void* dedup_workspace,
                           size_t dedup_workspace_bytes, uint8_t* keep, int* totals_written, void* stream);

/* The keyed step's record prep and text in ONE pass (round 6; the SoA read once):
 * what avdb_record_prep_keyed followed by avdb_primary_keys_onepass_ex compute —
 * end_out, bin_code, status (nullable); hist_l8 / counters accumulated (nullable); with
 * a K4 workspace (nullable) K4's long-record codes (then avdb_vrs_digest_ex with
 * AVDB_DIGEST_CODES_READY); with a K3 list workspace and keep (nullable) K3's first
 * phase (then avdb_pk_dedup_ex with AVDB_DEDUP_MARKED | AVDB_DEDUP_ONEPASS); and the
 * keys, ltree paths (path_out nullable: none), key_off[n+1] / path_off[n+1] and
 * key_state exactly as avdb_primary_keys_onepass_ex with digest == NULL (flags:
 * AVDB_KEYS_DIGEST_DEFERRED lays long keys out for avdb_primary_keys_fill_digests;
 * without it they are AVDB_KEY_NEED_DIGEST).  Text capacities as
 * avdb_primary_keys_bound.  workspace: avdb_keyed_prep_workspace_size(n) bytes,
 * 16-byte aligned (48 B per group of 1,024 records).  Groups of 256 records take their text
 * offsets from a decoupled look-back in the launch; *written = AVDB_KEYED_LONG_CODES |
 * AVDB_KEYED_DEDUP_MARKS for what it wrote.  avdb_keyed_prep_lookback_errors reads
 * (synchronously) how many look-back polls gave up in the last call on this workspace
 * (0 always expected; non-zero means its offsets are not valid). */
int avdb_keyed_prep_workspace_size(size_t n, size_t* bytes);
int avdb_keyed_prep(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                    const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                    const uint64_t* ext_id, size_t n, uint32_t max_seq_len, uint32_t* end_out, uint32_t* bin_code,
                    uint8_t* status, uint32_t* hist_l8, uint64_t* counters, void* workspace, size_t workspace_bytes,
                    void* digest_workspace, size_t digest_workspace_bytes, void* dedup_workspace,
                    size_t dedup_workspace_bytes, uint8_t* keep, uint64_t* key_off, uint64_t* path_off,
                    uint8_t* key_out, size_t key_cap, uint8_t* path_out, size_t path_cap, uint8_t* key_state,
                    uint32_t flags, int* written, void* stream);
int avdb_keyed_prep_lookback_errors(avdb_ctx* ctx, const void* workspace, uint32_t* out);

/* ---- K8: the per-record drop-in path in one launch -------------------------
 * The reference calls its per-record API once per alt allele
 * (vcf_variant_loader.py:282-311: __generate_primary_key, infer_variant_end_location,
 * find_bin_index, get_display_attributes).  For a small batch (one VCF line, one
 * find_bin_index miss) this entry does K2 + K7 + K5a in ONE launch of one
 * workgroup; every array may live in host-mapped pinned memory (avdb_host_alloc),
 * so a call is one launch + one stream sync, no copies.
 * Inputs: chrom, pos, and either end_in (bin of [pos, end_in]) or the alleles
 * (allele_off/ref_len/alt_len/heap, ext_id nullable: end inferred).  Outputs:
 * end_out, code, status per record; with alleles key_state (AVDB_KEY_*) and
 * disp_state (0 ok, 1 non-ASCII, 2 heap overrun); text streams selected by `want`
 * (AVDB_SMALL_PATH / _KEY / _DISPLAY) into text_out[k] (8-byte aligned, text_cap[k]
 * bytes) with offsets off_out[k*(n+1) + i] (u32).  A stream whose total exceeds
 * its cap is not written and sets bit k of *overflow. */
#define AVDB_SMALL_PATH 1u
#define AVDB_SMALL_KEY 2u
#define AVDB_SMALL_DISPLAY 4u
#define AVDB_SMALL_MAX 65536
typedef struct avdb_small_batch {
  const uint8_t* chrom;
  const uint32_t* pos;
  const uint32_t* end_in;
  const uint64_t* allele_off;
  const uint32_t* ref_len;
  const uint32_t* alt_len;
  const uint8_t* heap;
  const uint64_t* ext_id;
  size_t heap_bytes;
  uint32_t n;
  uint32_t max_seq_len;
  uint32_t want;
  uint32_t reserved;
  uint32_t* end_out;
  uint32_t* code;
  uint8_t* status;
  uint8_t* key_state;
  uint8_t* disp_state;
  uint32_t* off_out;
  uint8_t* text_out[3];
  uint32_t text_cap[3];
  uint32_t* overflow;
} avdb_small_batch;
int avdb_small_prep(avdb_ctx* ctx, const avdb_small_batch* batch, void* stream);
/* K8h: the same outputs computed by the library's host code from the kernels'
 * own record arithmetic (infer_end / classify / bin_path / display_json are
 * compiled for both sides), for callers that arrive one record or one VCF line
 * at a time — BinIndex.find_bin_index (bin_index.py:59-75) and
 * VCFVariantLoader.parse_variant (vcf_variant_loader.py:351-391) — where a GPU
 * launch + stream sync would cost more than the reference's whole call.  All
 * arrays are host memory; no stream, no device.  A context made with
 * device = -1 suffices. */
int avdb_small_prep_host(const avdb_ctx* ctx, const avdb_small_batch* batch);
/* K1h: the bin code, status and ltree path of ONE interval [start, end] (end >=
 * start; swapped intervals get status END_BEFORE_START as in K1) on the host —
 * one BinIndex.find_bin_index cache miss (bin_index.py:43-56,75).  Returns the
 * path length written to out (host, no NUL), 0 when unmappable (code ==
 * AVDB_BIN_NONE, or a contig beyond the labelled 25), or AVDB_ERANGE. */
int avdb_bin_path_host(const avdb_ctx* ctx, uint8_t chrom, uint32_t start, uint32_t end, uint32_t* code,
                       uint8_t* status, char* out_host, size_t cap);
/* K8a: ONE VariantAnnotator (Util/lib/python/variant_annotator.py:21-241) on the
 * host, for the drop-in class the reference constructs per alt allele
 * (vcf_parser.py:225-231, vcf_variant_loader.py:309-311).  alleles = REF bytes
 * then ALT bytes (host).  end_rel = infer_variant_end_location - pos (:36-79,
 * relative, so the caller's integer position is never narrowed); lcp = the
 * common-prefix length __normalize_alleles trims (:82-121).  With want_display,
 * the get_display_attributes fields (:134-241): location_start / _end, the class,
 * and the display_allele then sequence_allele texts in text[0, display_bytes +
 * sequence_bytes) — state 0; state 1 when they are the caller's (a non-ASCII
 * allele, or coordinates leaving u32), 2 when not asked.  Returns 0, or
 * AVDB_ERANGE when the two texts exceed cap (their sizes are set). */
#define AVDB_VC_SNV 0          /* single nucleotide variant / SNV */
#define AVDB_VC_INVERSION 1    /* inversion / MNV */
#define AVDB_VC_SUBSTITUTION 2 /* substitution / MNV */
#define AVDB_VC_INDEL 3        /* indel / INDEL */
#define AVDB_VC_INDEL_DOWN 4   /* indel / INDEL (insertion downstream of POS) */
#define AVDB_VC_INSERTION 5    /* insertion / INS */
#define AVDB_VC_DUPLICATION 6  /* duplication / DUP */
#define AVDB_VC_DELETION 7     /* deletion / DEL */
typedef struct avdb_annotation {
  int32_t end_rel;
  uint32_t lcp;
  uint32_t location_start;
  uint32_t location_end;
  uint32_t variant_class;
  uint32_t display_bytes;
  uint32_t sequence_bytes;
  uint32_t state;
} avdb_annotation;
int avdb_annotate_host(const avdb_ctx* ctx, const uint8_t* alleles, uint32_t ref_len, uint32_t alt_len,
                       uint32_t pos, int want_display, avdb_annotation* out, char* text, size_t cap);
/* Pinned host memory mapped into the device address space (hipHostMalloc,
 * mapped + coherent): the same pointer is valid on the host and in kernels. */
int avdb_host_alloc(size_t bytes, void** ptr);
int avdb_host_free(void* ptr);

/* ---- K6: duplicate check against variants already loaded ---------------
 * Replaces VariantRecord.exists / SQL map_variants(id, firstHitOnly, checkAltVariants)
 * (Util/lib/python/database/variant.py:41,287-309) as used by --skipExisting
 * (vcf_variant_loader.py:284-291).  The existing rows' metaseq ids form a key
 * set: keys = concatenated bytes, key_off[n_keys+1] (device).  build fills a
 * table of avdb_keyset_workspace_size(n_keys) bytes; probe writes per record
 * match[i] = index of the first equal key or -1, and kind[i]: */
#define AVDB_MATCH_NONE 0
#define AVDB_MATCH_EXACT 1              /* chrom:pos:ref:alt */
#define AVDB_MATCH_SWITCHED 2           /* chrom:pos:alt:ref (check_alt) */
#define AVDB_MATCH_HOST 255             /* contig without a canonical label: caller resolves */
int avdb_keyset_workspace_size(size_t n_keys, size_t* bytes);
int avdb_keyset_build(avdb_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, size_t n_keys, void* table,
                      size_t table_bytes, void* stream);
int avdb_keyset_probe(avdb_ctx* ctx, const void* table, size_t table_bytes, const uint8_t* keys,
                      const uint64_t* key_off, size_t n_keys, const uint8_t* chrom, const uint32_t* pos,
                      const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                      const uint8_t* heap, size_t heap_bytes, size_t n, int check_alt, int32_t* match,
                      uint8_t* kind, uint64_t* counters, void* stream);
/* The same key set probed with arbitrary strings q[q_off[i] .. q_off[i+1]) (device),
 * e.g. the primary keys avdb_primary_keys rendered: ADSP loads check each record's
 * primary key against the rows already loaded (is_duplicate(recordPK),
 * vcf_variant_loader.py:303-307).  match[i] = first equal key or -1; rows with
 * skip[i] != 0 (nullable) are not probed (-1). */
int avdb_keyset_probe_text(avdb_ctx* ctx, const void* table, size_t table_bytes, const uint8_t* keys,
                           const uint64_t* key_off, size_t n_keys, const uint8_t* q, const uint64_t* q_off,
                           const uint8_t* skip, size_t n, int32_t* match, uint64_t* counters, void* stream);

/* ---- K9: genome-piece sharding of VCF text --------------------------------
 * The reference runs one process per chromosome file (Load/bin/load_vcf_file.py:
 * 307-313).  One file is split over the ranks of a node by a piece plan
 * (annotatedvdb_amd/shard.py: contigs cut at `cut` bp, pieces assigned to ranks):
 * piece_base[c] / piece_count[c] (host, one per contig) index piece_rank[]
 * (host, n_pieces <= 1024).  A K0 data line belongs to the rank owning the piece
 * that holds its POS (a POS past the contig end: its last piece); lines K0 could
 * not place (host-resolved CHROM/POS, empty or short lines) belong to rank 0;
 * comment lines to none.
 *   avdb_vcf_select_lines: sel_off[n_lines+1] = exclusive scan of this rank's
 *     bytes per line (line length + 1), total in sel_off[n_lines]; workspace of
 *     avdb_shard_workspace_size(n_lines) bytes.
 *   avdb_vcf_select_copy:  the rank's lines, each + '
', into out (sel_off[n_lines]
 *     bytes), in file order. */
int avdb_shard_workspace_size(size_t n_lines, size_t* bytes);
int avdb_vcf_select_lines(avdb_ctx* ctx, size_t n_lines, const avdb_vcf_line* lines,
                          const uint32_t* piece_base_host, const uint32_t* piece_count_host,
                          const uint8_t* piece_rank_host, uint32_t n_pieces, uint32_t cut, int rank,
                          void* workspace, size_t workspace_bytes, uint64_t* sel_off, void* stream);
int avdb_vcf_select_copy(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                         const avdb_vcf_line* lines, const uint64_t* sel_off, uint8_t* out, void* stream);

/* ---- node exchange over RCCL (SURVEY.md §8b avdb_hist_allgather, §8e) ------
 * The one collective of the path: every rank's L8 histogram (u32[n_bins], the
 * hist_l8 K1/K2 accumulate) and counters (u64[n_counters]) all-gathered in one
 * RCCL call (xGMI inside a node) and summed over the ranks on the device into
 * node_hist / node_counters.  The reference has no collective (one process per
 * chromosome file, Load/bin/load_vcf_file.py:307-313).  Rank 0 makes the id
 * with avdb_rccl_unique_id, hands its AVDB_RCCL_ID_BYTES bytes to the other
 * ranks out of band, and every rank calls avdb_rccl_comm_init with its rank.
 * RCCL is loaded at first use (dlopen); these calls return AVDB_ERCCL when it
 * is absent.  Workspace: avdb_hist_allgather_workspace_size, 8-byte aligned. */
#define AVDB_RCCL_ID_BYTES 128
int avdb_rccl_unique_id(void* id);
int avdb_rccl_comm_init(avdb_ctx* ctx, int world, int rank, const void* id, void** comm);
int avdb_rccl_comm_destroy(void* comm);
int avdb_hist_allgather_workspace_size(int world, size_t n_bins, size_t n_counters, size_t* bytes);
int avdb_hist_allgather(avdb_ctx* ctx, void* comm, const uint32_t* hist, size_t n_bins,
                        const uint64_t* counters, size_t n_counters, uint32_t* node_hist,
                        uint64_t* node_counters, void* workspace, size_t workspace_bytes, void* stream);

/* ---- host-side formatting of kernel outputs -------------------------------
 * ltree path text (<= AVDB_MAX_PATH bytes).  Returns the length written (no
 * NUL terminator counted; one is written if cap allows), or a negative code. */
int avdb_format_bin_path(const avdb_ctx* ctx, uint8_t chrom, uint32_t bin_code, char* out_host,
                         size_t cap);
/* Batch form (host arrays): paths concatenated into out_host, out_off[i] the
 * start of path i, out_off[n] the total; returns AVDB_ERANGE if cap is short. */
int avdb_format_bin_paths(const avdb_ctx* ctx, const uint8_t* chrom_host, const uint32_t* code_host,
                          size_t n, char* out_host, size_t cap, uint64_t* out_off_host);

#ifdef __cplusplus
}
#endif
#endif /* AVDB_H_ */
