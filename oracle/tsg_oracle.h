/*
 * tsg_oracle.h — CPU ORACLE for the Tempo search path.  TEST INFRASTRUCTURE ONLY.
 *
 * A single-threaded-per-block, literal C restatement of the reference Go code
 * (Grafana Tempo ~v1.4.1, mounted at /root/reference) used as the parity
 * checker and as bench.py's cpu_baseline. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product (libtsg) never links,
 * calls or falls back to it.
 *
 * Parity pinning: the restatement is checked against the reference's own
 * fixtures and known-answer tests (tests/golden/): the v2test
 * block (bloom, index checksum, snappy pages, objects), TestContainsTag,
 * TestPipelineMatches{Tags,TraceDuration,TraceStartEnd,Block},
 * TestBackendSearchBlockSearch and TestStreamingSearchBlockSearchBlock metrics.
 * Flatbuffer page bytes written by the engine's own writer have no reference
 * golden (the reference commits none): read-back semantics are pinned, the
 * writer's byte layout is "parity unpinned".
 */
#ifndef TSG_ORACLE_H
#define TSG_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as tsg_request (tempopb.SearchRequest). */
typedef struct orc_request {
  uint32_t ntags;
  const uint8_t *const *tag_keys;
  const uint32_t *tag_key_lens;
  const uint8_t *const *tag_values;
  const uint32_t *tag_value_lens;
  uint32_t min_duration_ms, max_duration_ms, limit, start, end;
} orc_request;

typedef struct orc_match {
  uint8_t id[16]; /* right aligned */
  uint32_t id_len;
  uint32_t block_idx;
  uint64_t entry_idx;
  uint64_t start_ns, end_ns;
  uint32_t duration_ms;
  uint32_t svc_off, svc_len, name_off, name_len; /* into orc_result.strings */
} orc_match;

typedef struct orc_metrics {
  uint32_t traces_inspected, blocks_inspected, blocks_skipped, pad;
  uint64_t bytes_inspected;
} orc_metrics;

typedef struct orc_result {
  uint64_t n;
  orc_match *m;
  char *strings;
  uint64_t strings_len;
  orc_metrics metrics;
  int32_t status; /* first per-block error, 0 ok */
  int32_t pad;
  uint64_t nblocks;      /* orc_search: one status per block (the error its Search returned, 0 ok) */
  int32_t *block_status;
} orc_result;

typedef struct orc_block orc_block; /* search block files held in memory */

/* errors */
#define ORC_OK 0
#define ORC_NOT_FOUND 1
#define ORC_CORRUPT 2
#define ORC_UNSUPPORTED_ENCODING 3
#define ORC_INVALID 7
#define ORC_IO 9

int orc_block_load(const char *dir, orc_block **out);
/* search only index records [first_page, first_page + npages) (npages 0 = to the end) */
void orc_block_set_pages(orc_block *b, uint32_t first_page, uint32_t npages);
/* A search WAL file "<blockID>:<tenant>:v2:<encoding>[:...]" (StreamingSearchBlock):
 * orc_search replays it (header, sort, dedupe/combine) and searches it. */
int orc_wal_block_load(const char *path, orc_block **out);
/* Live traces (instance.searchLiveTraces, modules/ingester/instance_search.go:83-130):
 * segment i = bytes[seg_off[i], seg_off[i+1]) (a SearchEntry flatbuffer as pushed),
 * trace t = segments [trace_seg[t], trace_seg[t+1]) (a trace may have none). orc_search
 * matches every segment on its own and combines a trace's matches (CombineSearchResults);
 * entry_idx = the trace's position; no block filter, no blocksInspected. */
int orc_live_block_load_mem(const uint8_t *bytes, const uint64_t *seg_off, uint64_t nsegs, const uint64_t *trace_seg,
                            uint32_t ntraces, orc_block **out);
void orc_block_free(orc_block *b);
uint64_t orc_block_bytes(const orc_block *b);

/* BackendSearchBlock.Search over blocks in order, consumer = deterministic
 * refinement of instance.Search (limit 0 = every match). nthreads > 1 runs
 * one thread per block (only valid with limit 0; same result). */
int orc_search_seeded(orc_block *const *blocks, uint32_t nblocks, const orc_request *req, uint32_t limit,
                      const uint8_t (*seen)[16], uint64_t nseen, orc_result **out);
int orc_search(orc_block *const *blocks, uint32_t nblocks, const orc_request *req, uint32_t limit,
               int nthreads, orc_result **out);
int orc_combine(const orc_result *in, uint32_t max_results, orc_result **out);
void orc_result_free(orc_result *r);

/* Pipeline on single flatbuffers (pipeline_test.go). */
int orc_pipeline_matches_entry(const orc_request *req, const uint8_t *fb, size_t len);
int orc_pipeline_matches_block(const orc_request *req, const uint8_t *fb, size_t len);
int orc_contains_tag_entry(const uint8_t *fb, size_t len, const uint8_t *k, size_t kl,
                           const uint8_t *v, size_t vl);

/* Tags / TagValues of one block (backend: search-header, backend_search_block.go:145-181;
 * WAL: the replayed mutable header, streaming_search_block.go:97-116; live: every segment,
 * instance_search.go:187-240) and the instance aggregation (live blocks first, then the
 * others in order; TagValues' MapSizeWithinLimit check after each, max_bytes < 0 = off).
 * Output: sorted unique strings, u32 len + bytes each (malloc'd; orc_free). A backend block
 * without search data -> ORC_NOT_FOUND (readSearchHeader fails). */
int orc_block_tags(const orc_block *b, uint8_t **out, size_t *len, size_t *n);
int orc_block_tag_values(const orc_block *b, const uint8_t *key, size_t kl, uint8_t **out, size_t *len, size_t *n);
int orc_search_tags(orc_block *const *blocks, uint32_t nblocks, uint8_t **out, size_t *len, size_t *n);
int orc_search_tag_values(orc_block *const *blocks, uint32_t nblocks, const uint8_t *key, size_t kl, int64_t max_bytes,
                          uint8_t **out, size_t *len, size_t *n);

/* hashes */
uint64_t orc_xxhash64(const uint8_t *p, size_t n);
uint32_t orc_fnv1_32(const uint8_t *p, size_t n);
void orc_murmur3_128(const uint8_t *p, size_t n, uint64_t out[2]);
uint32_t orc_crc32c(const uint8_t *p, size_t n);
/* snappy framed stream -> out (malloc'd). */
int orc_snappy_framed_decode(const uint8_t *src, size_t n, uint8_t **out, size_t *out_len);

/* v2 trace blocks */
typedef struct orc_v2block orc_v2block;
int orc_v2block_load(const char *dir, orc_v2block **out);
void orc_v2block_free(orc_v2block *b);
/* bloom.Test for the shard the id maps to: 1/0, <0 error */
int orc_v2_bloom_test(const orc_v2block *b, const uint8_t *id, size_t idlen);
/* indexReader.Find: record index (or -1), record fields */
int orc_v2_index_find(const orc_v2block *b, const uint8_t *id, size_t idlen, int64_t *rec_idx,
                      uint64_t *start, uint32_t *length);
/* BackendBlock.find: object bytes (malloc'd) or *out=NULL when absent */
int orc_v2_find(const orc_v2block *b, const uint8_t *id, size_t idlen, uint8_t **out,
                size_t *out_len);
/* includeBlock (tempodb.go:492-511); time window both 0 = off; range NULL = off */
int orc_v2_include_block(const orc_v2block *b, const uint8_t *id, uint32_t ts, uint32_t te,
                         const uint8_t *bstart, const uint8_t *bend);
/* Batched lookup = tsg_lookup_ids semantics: hits sorted (id_idx, block_idx). */
typedef struct orc_hit {
  uint32_t id_idx, block_idx;
  int32_t record_idx;
  uint32_t record_length;
  uint64_t record_start;
} orc_hit;
int orc_lookup_ids(orc_v2block *const *blocks, uint32_t nblocks, const uint8_t (*ids)[16],
                   uint64_t nids, uint32_t ts, uint32_t te, const uint8_t *bstart,
                   const uint8_t *bend, int nthreads, orc_hit **out, uint64_t *nout);
uint32_t orc_v2_shard_count(const orc_v2block *b);

void orc_free(void *p);

/* CPU columnar baseline (bench.py cpu_baseline.columnar; SURVEY.md §8(d) "CPU columnar"
 * variant): a backend search block decoded once into host columns (start/end ns, and
 * per key the KeyValues value-set id of every entry), then the Pipeline predicates
 * evaluated over the columns, multi-threaded over entries. Same match set as the
 * reference's scan for backend blocks (unique keys per entry); it is a baseline to time,
 * not a restatement. */
typedef struct orc_colblock orc_colblock;
int orc_colblock_build(const orc_block *b, orc_colblock **out);
void orc_colblock_free(orc_colblock *c);
uint64_t orc_colblock_entries(const orc_colblock *c);
/* matches of req over the blocks (limit ignored: full scan); *hash = sum over matches of
 * (block index << 32 | scan position) * golden-ratio constant (order independent) */
int orc_columnar_search(orc_colblock *const *cbs, uint32_t n, const orc_request *req, int nthreads,
                        uint64_t *matches, uint64_t *hash);
/* SearchEntryMutable.ToBytes (Go flatbuffers builder restatement); *out malloc'd */
int orc_entry_to_bytes(const uint8_t *id, size_t idl, uint64_t st, uint64_t en, uint32_t npairs,
                       const uint8_t *const *k, const uint32_t *kl, const uint8_t *const *v, const uint32_t *vl,
                       uint8_t **out, size_t *out_len);

#ifdef __cplusplus
}
#endif
#endif
