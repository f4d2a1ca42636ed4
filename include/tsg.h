/*
 * tsg.h — C ABI of libtsg, the MI355X (gfx950) Tempo search engine.
 *
 * This is the drop-in boundary for Tempo's flatbuffer backend-search path and the
 * v2 trace-ID lookup path. Every entry point takes plain pointers and sizes; no
 * Go, Python or torch types cross it. All inputs are copied during the call and
 * no caller pointer is retained (cgo rule: C may not keep Go pointers).
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference checkout, Grafana Tempo ~v1.4.1):
 *
 *   tsg_block_open        search.OpenBackendSearchBlock + the reads at the top of
 *                         BackendSearchBlock.Search
 *                         (tempodb/search/backend_search_block.go:132-138,184-241)
 *   tsg_search            BackendSearchBlock.Search page/entry loops driven by
 *                         instance.searchLocalBlocks
 *                         (tempodb/search/backend_search_block.go:247-295,
 *                          modules/ingester/instance_search.go:164-185)
 *   tsg_pipeline_new      search.NewSearchPipeline + rewriteTagLookup
 *                         (tempodb/search/pipeline.go:26-140)
 *   tsg_results_combine   the consumer loop of instance.Search
 *                         (modules/ingester/instance_search.go:45-70) with
 *                         search.CombineSearchResults (tempodb/search/util.go:40-62)
 *   tsg_block_tags /      BackendSearchBlock.Tags / TagValues
 *   tsg_block_tag_values  (tempodb/search/backend_search_block.go:145-181),
 *                         StreamingSearchBlock.Tags / TagValues
 *                         (tempodb/search/streaming_search_block.go:97-116)
 *   tsg_search_tags /     instance.SearchTags / SearchTagValues
 *   tsg_search_tag_values (modules/ingester/instance_search.go:187-273)
 *   tsg_live_block_open_mem  the live traces instance.searchLiveTraces walks
 *                         (modules/ingester/instance_search.go:83-130), searched by
 *                         tsg_search like any other block
 *   tsg_v2block_open /    v2.BackendBlock.find: bloom shard select + bloom test +
 *   tsg_lookup_ids        index lower_bound (tempodb/encoding/v2/backend_block.go:38-92,
 *                         tempodb/encoding/common/bloom.go:83-93,
 *                         tempodb/encoding/v2/index_reader.go:85-114) and the
 *                         tempodb.Find block prefilter (tempodb/tempodb.go:492-511)
 *
 * Threading: a tsg_ctx is thread-safe. Blocks on different devices are searched in
 * parallel. On one device, narrow searches from concurrent callers (and the items of
 * tsg_search_batch) are in flight together: each is posted to the device's resident search
 * kernel while earlier ones run, and the kernel serves them back to back (up to
 * TSG_RES_DEPTH at once); other searches on the device are serialised on its stream.
 *
 * Errors: every int-returning call returns a TSG_* status; tsg_last_error()
 * returns the thread-local message of the last failure on this thread.
 */
#ifndef TSG_H
#define TSG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSG_ABI_VERSION 7

/* Status codes. */
#define TSG_OK 0
#define TSG_E_NOT_FOUND 1            /* search.meta.json missing: the Go shim maps this to a no-op
                                        (backend_search_block.go:191-203) */
#define TSG_E_CORRUPT 2              /* checksum / offset / framing error */
#define TSG_E_UNSUPPORTED_ENCODING 3 /* search_encoding other than none/snappy, or version != v2 */
#define TSG_E_DEVICE 4               /* HIP runtime failure or no device */
#define TSG_E_CANCELLED 5
#define TSG_E_OOM 6
#define TSG_E_INVALID 7              /* bad argument */
#define TSG_E_UNSUPPORTED 8          /* block layout outside the engine's contract */
#define TSG_E_IO 9

typedef struct tsg_ctx tsg_ctx;
typedef struct tsg_block tsg_block;
typedef struct tsg_pipeline tsg_pipeline;
typedef struct tsg_v2block tsg_v2block;

typedef struct tsg_options {
  int32_t num_devices;    /* 0 = every visible device */
  const int32_t *devices; /* optional explicit ordinals (num_devices entries) */
  uint32_t flags;         /* reserved, 0 */
} tsg_options;

/* tempopb.SearchRequest (pkg/tempopb/tempo.proto:44-52), un-normalised. */
typedef struct tsg_request {
  uint32_t ntags;
  const uint8_t *const *tag_keys;
  const uint32_t *tag_key_lens;
  const uint8_t *const *tag_values;
  const uint32_t *tag_value_lens;
  uint32_t min_duration_ms;
  uint32_t max_duration_ms;
  uint32_t limit;
  uint32_t start; /* unix seconds */
  uint32_t end;   /* unix seconds */
} tsg_request;

/* The normalised query a Pipeline applies: what the Go shim passes after
 * rewriteTagLookup + strings.ToLower (tempodb/search/pipeline.go:26-101). */
typedef struct tsg_query {
  uint32_t nterms;
  const uint8_t *const *keys;
  const uint32_t *key_lens;
  const uint8_t *const *values;
  const uint32_t *value_lens;
  uint8_t has_min;    /* MinDurationMs > 0 */
  uint8_t has_max;    /* MaxDurationMs > 0 */
  uint8_t has_range;  /* Start != 0 && End != 0 */
  uint8_t exhaustive; /* x-dbg-exhaustive: always-false trace filter */
  uint64_t min_ns;
  uint64_t max_ns;
  uint32_t start_s;
  uint32_t end_s;
} tsg_query;

/* tempopb.SearchMetrics (pkg/tempopb/tempo.proto:81-87) + device counters. */
typedef struct tsg_metrics {
  uint32_t traces_inspected;
  uint32_t blocks_inspected;
  uint32_t blocks_skipped;
  uint32_t reruns;            /* extra search-kernel launches (a workgroup's records overflowed
                                 its buffer); their device time is in kernel_ns / scan_kernel_ns */
  uint64_t bytes_inspected;
  uint64_t device_bytes_read; /* algorithmic bytes the scan kernels touched */
  uint64_t kernel_ns;         /* device time of the search kernels (HIP events) */
  uint64_t scan_kernel_ns;    /* device time of the scan_compact kernel alone (HIP events) */
  uint64_t scan_bytes;        /* algorithmic bytes of the scan_compact kernel */
  /* ABI 7: the kernels that served this search (TSG_PATH_* bits, OR over devices, chunks and
     limit waves). TSG_PATH_COTENANT: the resident kernel was passed over because another process
     has a libtsg context on the same GPU (its launch would hold every CU). */
  uint32_t path;
  uint32_t reserved;
} tsg_metrics;
#define TSG_PATH_RESIDENT 1u /* search_resident_kernel (narrow query, mailbox) */
#define TSG_PATH_PLAIN 2u    /* search_pool_kernel / search_static_kernel as plain launches */
#define TSG_PATH_OTHER 4u    /* search_fast_kernel, the dictionary pass, the general path */
#define TSG_PATH_COTENANT 8u /* the resident kernel declined: another process on the GPU */

/* Ordered match sequence: blocks in caller order, each block's matches in the
 * reference scan order (pages ascending, entry vector index ascending). With
 * limit L > 0 the sequence is cut right after the first occurrence of the L-th
 * distinct trace ID (deterministic refinement of instance.Search). */
typedef struct tsg_result {
  uint64_t n;
  const uint8_t (*trace_id)[16]; /* right-aligned, zero-padded on the left */
  const uint8_t *trace_id_len;   /* original id length (<= 16) */
  const uint64_t *start_ns;
  const uint64_t *end_ns;
  const uint32_t *duration_ms; /* uint32((end-start)/1e6), util.go:33 */
  const uint32_t *block_idx;   /* index into the caller's block array */
  const uint64_t *entry_idx;   /* scan position inside the block */
  const char *const *root_service; /* (not NUL-terminated) lengths below */
  const uint32_t *root_service_len;
  const char *const *root_name;
  const uint32_t *root_name_len;
  tsg_metrics metrics;
  /* Per caller block (nblocks entries): TSG_OK, or the error the reference's
   * BackendSearchBlock.Search returns for that block AFTER the matches listed above
   * (a damaged data page, backend_search_block.go:258-266; the ingester logs it and
   * keeps the other blocks' results, instance_search.go:179-182). block_error[i] is
   * the message (NULL when OK). A damaged index ends a block silently instead
   * (`record, _ := ir.At(ctx, i)`, :252-255): no error, fewer pages. */
  uint64_t nblocks;
  const int32_t *block_status;
  const char *const *block_error;
  /* Every name above as one blob: root_service[i] == names + root_service_off[i] (likewise
   * root_name). Equal names of one dictionary share their bytes, so a dense result's blob
   * stays small; a packed transport (tempo_amd/shard.py) ships it as it is. */
  const char *names;
  uint64_t names_len;
  const uint64_t *root_service_off;
  const uint64_t *root_name_off;
} tsg_result;

/* Options for tsg_search. */
#define TSG_SEARCH_TIME_SCAN 1u /* HIP events around the scan kernel -> metrics.scan_kernel_ns */
#define TSG_SEARCH_TIME_ALL 2u  /* ... and around the whole device sequence -> metrics.kernel_ns */
#define TSG_SEARCH_TIME_DEFER 4u /* HIP events around the search kernel, read later with
                                    tsg_kernel_times (the search does not wait for them) */
typedef struct tsg_search_opts {
  uint32_t limit;  /* 0 = no limit (every match) */
  uint32_t flags;  /* TSG_SEARCH_TIME_* (timing events cost a few us per search; off by default) */
  uint64_t query_id; /* for tsg_cancel; 0 = not cancellable. tsg_cancel on an id while its search
                        runs stops it at the next device chunk or wave (TSG_E_CANCELLED); a cancel
                        for an id whose search finished recently is ignored (it cannot fail a later
                        search that reuses the id); one for an id not seen yet waits up to 10 s for
                        its search to start. */
  /* ABI 5: trace IDs the caller's consumer has already taken (16 bytes each, right-aligned
     like tsg_result.trace_id), counted toward `limit` as if they had been consumed first:
     the search stops where a consumer that saw them before this call's blocks stops. A
     querier fanning blocks out over ranks (modules/frontend/searchsharding.go:88-106,
     tempo_amd/shard.py distributed_search_limit) passes the distinct IDs of the blocks
     before this rank's. NULL / 0 = none. */
  const uint8_t (*seen_ids)[16];
  uint64_t nseen;
} tsg_search_opts;

/* ---- context --------------------------------------------------------------- */
int tsg_init(const tsg_options *opts, tsg_ctx **out);
void tsg_shutdown(tsg_ctx *ctx);
int tsg_device_count(tsg_ctx *ctx);
/* NUMA node of device `dev`'s PCI function (sysfs), -1 if unknown. The search path
 * polls a completion word and reads its records in pinned host memory: a caller that
 * keeps its search threads on this node's CPUs sees both sooner. */
int tsg_device_numa_node(tsg_ctx *ctx, int dev);
/* ABI 6: the device context's resident-search counters, out[0..n): [0] resident launches,
 * [1] queries they served, [2] relaunches after a launch left on its idle timeout as a query
 * was posted, [3] quits (another kernel needed the device, a second context opened on it, or
 * the query shape changed). ABI 7: [4] mailbox slot reads the kernel rejected (check mismatch:
 * a read that caught the host's writes landing), [5] narrow queries launched plainly because
 * another process has a libtsg context on the same GPU, [6] narrow queries launched plainly
 * (any reason), [7] samples taken for the XCD-weighted split. Zeros when TSG_RESIDENT=0.
 * DESIGN.md §4. */
int tsg_device_counters(tsg_ctx *ctx, int dev, uint64_t *out, size_t n);
const char *tsg_last_error(void);
int tsg_abi_version(void);
int tsg_cancel(tsg_ctx *ctx, uint64_t query_id);

/* ---- pipeline (request normalisation, host) ---------------------------------- */
int tsg_pipeline_new(const tsg_request *req, tsg_pipeline **out);
const tsg_query *tsg_pipeline_query(const tsg_pipeline *p);
void tsg_pipeline_free(tsg_pipeline *p);
/* Pipeline.MatchesBlock on a raw search-header flatbuffer (pipeline.go:172-183). */
int tsg_pipeline_matches_header(const tsg_query *q, const uint8_t *header, size_t len,
                                int *matches);

/* ---- backend search blocks ------------------------------------------------------ */
/* Reads <block_dir>/{search.meta.json,search-header,search-index,search}, validates
 * checksums and framing, decodes every page once into the device-resident
 * columnar layout on device (device_hint % devices). */
int tsg_block_open(tsg_ctx *ctx, const char *block_dir, int device_hint, tsg_block **out);
/* ABI 6: one page range of a block — index records [first_page, first_page + npages), npages
 * past the end = to the end — as its own resident block. The frontend splits a large block
 * into jobs of whole pages sized by bytes (StartPage / PagesToSearch of a SearchBlockRequest,
 * modules/frontend/searchsharding.go:325-367); tempo_amd.shard.plan_shards does the same to
 * balance blocks over ranks. A range's search applies the block's header filter; a range that
 * does not start at page 0 counts neither the header's bytes nor the block as inspected or
 * skipped, so the ranges of a block sum to the block's metrics. Scan positions (entry_idx)
 * are inside the range. */
int tsg_block_open_pages(tsg_ctx *ctx, const char *block_dir, uint32_t first_page, uint32_t npages,
                         int device_hint, tsg_block **out);
/* Same from caller buffers (copied). meta_json may be NULL -> TSG_E_NOT_FOUND. */
int tsg_block_open_mem(tsg_ctx *ctx, const uint8_t *meta_json, size_t meta_len,
                       const uint8_t *header, size_t header_len, const uint8_t *index,
                       size_t index_len, const uint8_t *data, size_t data_len, int device_hint,
                       tsg_block **out);
void tsg_block_close(tsg_block *b);
/* A second resident copy of an open block (backend or WAL) on device_hint's device:
 * device-to-device copies of its columns and dictionaries. Replicates a block onto
 * another GPU without re-reading and re-decoding its files (block-sharded serving with
 * replicas), or makes disjoint copies of one data set (bench.py's HBM-regime rotation). */
int tsg_block_clone(tsg_ctx *ctx, const tsg_block *src, int device_hint, tsg_block **out);

/* ---- WAL search blocks (StreamingSearchBlock) -------------------------------------- */
/* Replaces search.RescanBlocks' per-file replay + StreamingSearchBlock.Search's
 * iterator (tempodb/search/rescan_blocks.go:74-107, streaming_search_block.go:118-237):
 * path names a search WAL file "<blockID>:<tenant>:v2:<encoding>[:<dataEncoding>]"
 * (wal.ParseFilename, tempodb/wal/wal.go:179-219). Pages are replayed in file order (the
 * block header is SearchBlockHeaderMutable over every page), records sorted by id,
 * equal ids combined (DataCombiner), and the entries become one resident block; a
 * damaged page ends the replay (tsg_block_info.partial). An empty file ->
 * TSG_E_NOT_FOUND (RescanBlocks drops it). The handle is searched with tsg_search like
 * a backend block: block filter on the mutable header (exact-value tag Contains),
 * bytesInspected = object bytes of the entries visited, no header bytes. */
int tsg_wal_block_open(tsg_ctx *ctx, const char *path, int device_hint, tsg_block **out);
int tsg_wal_block_open_mem(tsg_ctx *ctx, const uint8_t *data, size_t len, int encoding, int device_hint,
                           tsg_block **out);

/* ---- live traces (instance.searchLiveTraces) -------------------------------------- */
/* A snapshot of the ingester's live traces (i.traces, in its iteration order), copied in:
 * segment i = bytes[seg_off[i], seg_off[i+1]) is one searchData buffer as the distributor
 * pushed it (a SearchEntry flatbuffer; liveTrace.searchData, modules/ingester/trace.go:37,76-80),
 * trace t owns segments [trace_seg[t], trace_seg[t+1]) (trace_seg[0] = 0, trace_seg[ntraces] =
 * nsegs; a trace without search data has none). tsg_search on the handle restates
 * searchLiveTraces (instance_search.go:83-130): every segment is matched on its own
 * (Pipeline.Matches), a trace's matching segments are combined with CombineSearchResults
 * (tempodb/search/util.go:40-62) into one result whose entry_idx is the trace's position;
 * tracesInspected += 1 per trace visited, bytesInspected += every segment's length; no block
 * filter, no blocksInspected. Under a limit the consumer stops after the trace that brings the
 * L-th distinct id (the deterministic refinement). A segment shorter than 4 bytes
 * -> TSG_E_CORRUPT (the reference's entry.Reset panics). */
int tsg_live_block_open_mem(tsg_ctx *ctx, const uint8_t *bytes, const uint64_t *seg_off, size_t nsegs,
                            const uint64_t *trace_seg, size_t ntraces, int device_hint, tsg_block **out);

typedef struct tsg_block_info {
  uint64_t entries;
  uint64_t pages;
  uint64_t keys;
  uint64_t header_bytes;
  uint64_t fb_bytes;       /* sum of flatbuffer page bytes (bytesInspected per full scan) */
  uint64_t device_bytes;   /* resident bytes on device */
  uint64_t min_dur_ns;     /* on-disk search-header values (pitfall P1) */
  uint64_t max_dur_ns;
  int32_t device;
  int32_t encoding;        /* backend.Encoding numeric value */
  int32_t streaming;       /* 1: a WAL (StreamingSearchBlock) replay */
  int32_t partial;         /* 1: the WAL replay stopped at a damaged page (the reference's warning) */
  int32_t stop_status;     /* backend block with a damaged data page: the error its Search returns
                              after the pages before it (0 = none) */
  int32_t index_truncated; /* 1: an index record failed (checksum, framing, zero record): the block
                              ends silently before it, as the reference's Search does */
  int32_t live;            /* 1: live traces (tsg_live_block_open_mem) */
  int32_t hdr_deferred;    /* ABI 6: header keys whose MatchesBlock value test comes from the device
                              dictionary pass (the header's values are the dictionary, compared
                              byte for byte at open) */
  uint64_t traces;         /* live: traces (entries = their segments); otherwise = entries */
} tsg_block_info;
int tsg_block_info_get(const tsg_block *b, tsg_block_info *out);

/* SearchableBlock.Tags / TagValues of one block: a backend block's search-header (Tags: every
 * key of the header rollup; TagValues: FindTag on it), a WAL block's mutable header (the
 * exact key's values), live traces (Tags: every key of every segment; TagValues: FindTag on
 * every segment). Output is a packed list, sorted and unique: u32 len + bytes, repeated;
 * *out_n = count. Free with tsg_free. A backend block opened without search data ->
 * TSG_E_NOT_FOUND (its readSearchHeader fails with ErrDoesNotExist). */
int tsg_block_tags(const tsg_block *b, uint8_t **out, size_t *out_len, size_t *out_n);
int tsg_block_tag_values(const tsg_block *b, const uint8_t *key, size_t klen, uint8_t **out,
                         size_t *out_len, size_t *out_n);
/* instance.SearchTags / SearchTagValues over an instance's searchable blocks: live blocks
 * first, then the others in caller order (WAL head + append blocks, then local blocks, as the
 * ingester visits them); the first block error fails the call. TagValues applies
 * util.MapSizeWithinLimit (sum of the distinct values' lengths < max_bytes) after the live
 * blocks and again after all blocks and returns an EMPTY list when it fails, as the reference
 * does to protect the querier (overrides MaxBytesPerTagValuesQuery, default 5e6);
 * max_bytes < 0 = no check. Same output format as tsg_block_tags. */
int tsg_search_tags(tsg_block *const *blocks, size_t nblocks, uint8_t **out, size_t *out_len, size_t *out_n);
int tsg_search_tag_values(tsg_block *const *blocks, size_t nblocks, const uint8_t *key, size_t klen,
                          int64_t max_bytes, uint8_t **out, size_t *out_len, size_t *out_n);
void tsg_free(void *p);

/* Search blocks[0..nblocks) with the normalised query. Blocks may live on
 * different devices; the result is the single ordered sequence described at
 * tsg_result. */
int tsg_search(tsg_ctx *ctx, tsg_block *const *blocks, size_t nblocks, const tsg_query *q,
               const tsg_search_opts *opts, tsg_result **out);
void tsg_result_free(tsg_result *r);

/* ABI 7: a batch of searches served back to back (SURVEY §8(d) batched mode; the ingester's
 * concurrent Search calls, modules/ingester/instance_search.go:164-185, in one call). Item i is
 * one tsg_search (its own blocks, query and options) whose result goes to outs[i] (free each with
 * tsg_result_free; NULL for a failed item). Up to `depth` items (0 = 16) run at once on internal
 * threads and skip the coalescer: a narrow query is posted to the resident kernel's mailbox while
 * earlier ones run, so the device serves them back to back. Returns TSG_OK or the first failing
 * item's status. device_ns (optional): when each device's resident queries of the batch ran on
 * one resident launch that this call started and ended, the longest such launch's dispatch
 * duration (the AQL queue's dispatch timestamps, the clock rocprofv3's kernel trace reads); 0
 * otherwise. */
typedef struct tsg_search_item {
  tsg_block *const *blocks;
  size_t nblocks;
  const tsg_query *query;
  tsg_search_opts opts;
} tsg_search_item;
int tsg_search_batch(tsg_ctx *ctx, const tsg_search_item *items, size_t n, uint32_t depth, tsg_result **outs,
                     uint64_t *device_ns);

/* ABI 7, test hooks (process-wide): "res_torn" = k: the next k resident-kernel posts write the
 * mailbox slot as a read that caught the host's writes half landed would see it (two argument
 * words moved by +-d: the plain sum unchanged) and repair it 200 us later; the kernel must
 * re-read the slot (tsg_device_counters[4] counts the rejected reads). "groups" = n (0 = the
 * device's CUs): search launches plan for n CUs. "xsplit" = 0/1: the resident kernel's
 * XCD-weighted split (default TSG_RES_XSPLIT, off). "lb_bitmap" = 0/1/2: full scans on the
 * dictionary-pass path return one bit per entry never / always / after a dense one (default
 * TSG_LB_BITMAP, 2). TSG_E_INVALID for an unknown name. */
int tsg_debug_set(const char *name, int64_t value);

/* Durations (ns) of the search kernels launched with TSG_SEARCH_TIME_DEFER since
 * the last call, in launch order per device (devices in context order). Waits for
 * every device's stream. At most cap values are written; *n = values written. */
int tsg_kernel_times(tsg_ctx *ctx, uint64_t *ns, size_t cap, size_t *n);

/* instance.Search consumer on an ordered match sequence: dedupe by trace ID with
 * CombineSearchResults, stop at max_results distinct (0 -> 20), then sort by
 * StartTimeUnixNano descending (ties: first scan position). Output has the same
 * layout as tsg_result (block_idx/entry_idx = first occurrence). */
int tsg_results_combine(const tsg_result *in, uint32_t max_results, tsg_result **out);

/* ---- multi-GPU fan-out: packed responses and the frontend merge ------------------ */
/* A response (one rank's / one job's tempopb.SearchResponse) as one byte buffer, for the
 * gather to the merging rank (tempo_amd/shard.py). Little endian, sections 8-byte aligned:
 *   tsg_wire_header | n x tsg_trace_rec | (nnames + 1) x u32 name offsets | names bytes |
 *   nblocks x i32 block status | errors (per block with a non-zero status, in block order:
 *   u32 length + message bytes)
 * A record's names are indices into the name table (entry 0 = ""). */
#define TSG_WIRE_MAGIC 0x57475354u /* "TSGW" */
#define TSG_WIRE_VERSION 1u
typedef struct tsg_trace_rec { /* tempopb.TraceSearchMetadata (pkg/tempopb/tempo.proto:72-79) */
  uint8_t trace_id[16];        /* right-aligned (hex TraceID = these bytes, leading zeros trimmed) */
  uint64_t start_ns;
  uint32_t duration_ms;
  uint32_t root_service; /* name table index */
  uint32_t root_name;
  uint8_t trace_id_len;
  uint8_t pad[3];
} tsg_trace_rec;
typedef struct tsg_wire_header {
  uint32_t magic, version;
  uint64_t n, nnames, names_len, nblocks, errors_len;
  uint64_t traces_inspected, bytes_inspected, blocks_inspected, blocks_skipped, skipped_traces; /* SearchMetrics */
  uint64_t reserved;
} tsg_wire_header;
/* A tsg_result as a wire buffer (malloc'd; tsg_free). */
int tsg_result_pack(const tsg_result *r, uint8_t **out, size_t *out_len);
/* searchResponse (modules/frontend/searchsharding.go:32-125) over wire responses in the given
 * order: before each response, shouldQuit (more than `limit` distinct traces taken) stops the
 * merge; addResponse keeps the first record of every TraceID and sums InspectedTraces /
 * InspectedBytes / SkippedBlocks / SkippedTraces; InspectedBlocks = total_blocks (set by the
 * sharder, :221); result sorts by start time descending (ties: first position, a deterministic
 * form of sort.Slice). Block statuses and errors of every response are carried in order. The
 * merged response is written as a wire buffer into the caller's `out` (cap bytes; for n >= 1
 * the sum of the input lengths always suffices, n = 0 needs sizeof(tsg_wire_header) + 8):
 * *out_len = its length; TSG_E_INVALID with *out_len = the needed size when cap is too small. Host code, no device needed; parallel over host threads. */
int tsg_wire_merge(const uint8_t *const *wires, const size_t *lens, size_t n, uint64_t limit, uint64_t total_blocks,
                   uint8_t *out, size_t cap, size_t *out_len);

/* ABI 7: the same merge for the ranks of one node through shared memory (/dev/shm/<name>): each
 * rank puts its wire for query `seq` (1, 2, ... in every rank's call order) into its slot;
 * rank 0's tsg_shm_merge waits for every rank's response to `seq` and merges them in place (as
 * tsg_wire_merge, ranks in order). Slots are double buffered: a rank may put query seq + 1
 * while rank 0 merges seq. Waits are bounded by timeout_s (TSG_E_DEVICE: a rank did not
 * answer). Rank 0 opens with reset = 1 before the others open (tempo_amd/shard.py ShmGather:
 * a barrier between); rank 0's close removes the file. A response above slot_bytes ->
 * TSG_E_INVALID (the caller gathers it another way). */
typedef struct tsg_shm tsg_shm;
int tsg_shm_open(const char *name, uint32_t world, uint32_t rank, uint64_t slot_bytes, int reset, tsg_shm **out);
void tsg_shm_close(tsg_shm *s);
int tsg_shm_put(tsg_shm *s, uint32_t seq, const uint8_t *wire, size_t len, double timeout_s);
int tsg_shm_merge(tsg_shm *s, uint32_t seq, uint64_t limit, uint64_t total_blocks, uint8_t *out, size_t cap,
                  size_t *out_len, double timeout_s);

/* ---- v2 trace blocks: batched trace-ID lookup --------------------------------- */
/* Reads <block_dir>/{meta.json,bloom-N...,index}; verifies index page checksums. */
int tsg_v2block_open(tsg_ctx *ctx, const char *block_dir, int device_hint, tsg_v2block **out);
void tsg_v2block_close(tsg_v2block *b);

typedef struct tsg_lookup_opts {
  uint32_t time_start; /* tempodb.Find window (unix s); both 0 = no time filter */
  uint32_t time_end;
  const uint8_t *block_start; /* 16-byte blockID shard range, NULL = no range */
  const uint8_t *block_end;
} tsg_lookup_opts;

/* One hit per (id, block) pair where includeBlock passes, bloom.Test is true
 * and the index lower_bound is < TotalRecords, sorted by (id_idx, block_idx).
 * Blocks may live on different devices: every device probes all ids against its own
 * blocks concurrently (tempodb.Find's per-block fan-out) and the lists are merged.
 * Exactly the (record, i) pairs the reference hands to findOne
 * (tempodb/encoding/v2/finder_paged.go:37-48); bloom false positives included. */
typedef struct tsg_lookup_result {
  uint64_t n;
  const uint32_t *id_idx;
  const uint32_t *block_idx;
  const int32_t *record_idx;
  const uint64_t *record_start;
  const uint32_t *record_length;
  uint64_t kernel_ns;
} tsg_lookup_result;

int tsg_lookup_ids(tsg_ctx *ctx, tsg_v2block *const *blocks, size_t nblocks,
                   const uint8_t (*ids)[16], size_t nids, const tsg_lookup_opts *opts,
                   tsg_lookup_result **out);
void tsg_lookup_result_free(tsg_lookup_result *r);

/* tempodb.Find's per-block step for a batch of ids, whole on the device: the lookup above,
 * then PagedFinder.findOne (tempodb/encoding/v2/finder_paged.go:79-110) for every hit: the
 * data page its index record names (resident in HBM since tsg_v2block_open) is decompressed
 * (encodings none, snappy and zstd; others -> TSG_E_UNSUPPORTED_ENCODING for that hit) and its
 * objects are scanned for the exact id. One entry per lookup hit, sorted (id_idx,
 * block_idx): status TSG_OK with the object's bytes (what findOne returns), TSG_E_NOT_FOUND
 * (a bloom false positive: findOne returns nil), or the error findOne returns for that
 * page (read, framing, decompression, object framing). */
typedef struct tsg_find_result {
  uint64_t n;
  const uint32_t *id_idx;
  const uint32_t *block_idx;
  const int32_t *status;
  const uint64_t *obj_off; /* into obj_bytes (status TSG_OK) */
  const uint32_t *obj_len;
  const uint8_t *obj_bytes;
  uint64_t kernel_ns;
} tsg_find_result;
int tsg_find_ids(tsg_ctx *ctx, tsg_v2block *const *blocks, size_t nblocks, const uint8_t (*ids)[16],
                 size_t nids, const tsg_lookup_opts *opts, tsg_find_result **out);
void tsg_find_result_free(tsg_find_result *r);

/* ---- proto-object backend search ---------------------------
 * tempodb.Search over one v2 block whose objects are trace protos: what querier and
 * serverless SearchBlock jobs run (modules/querier/querier.go:420-452 ->
 * tempodb/tempodb.go:368-375 -> v2.BackendBlock.Search, tempodb/encoding/v2/
 * backend_block.go:159-231 -> ObjectDecoder.Matches -> trace.MatchesProto,
 * pkg/model/trace/matches.go:33-184). meta.json dataEncoding "v1" (objects are
 * tempopb.TraceBytes) or "v2" (u32 start, u32 end seconds + TraceBytes, with the FastRange
 * and duration prefilter, pkg/model/v2/object_decoder.go:57-89). tsg_proto_block_open
 * decodes every data page (none, snappy, zstd) and every object once into per-object
 * columns and per-attribute-key value-set columns resident on the device; a search is one
 * kernel over the page range plus the host replay of Search's loop. */
typedef struct tsg_proto_block tsg_proto_block;
typedef struct tsg_proto_request {
  uint32_t ntags; /* SearchRequest.Tags (map: a repeated key keeps its last value) */
  const char *const *keys;
  const uint32_t *key_lens;
  const char *const *values;
  const uint32_t *value_lens;
  uint32_t min_duration_ms, max_duration_ms; /* 0 = unset */
  uint32_t start, end;                       /* unix seconds (compared even when 0, as the reference) */
  uint32_t limit;                            /* Search breaks once len(Traces) >= Limit (0: after one object) */
  uint32_t start_page, total_pages;          /* SearchOptions: total_pages > 0 = partial iterator */
  uint32_t max_bytes;                        /* SearchOptions.MaxBytes: larger objects are SkippedTraces */
  uint32_t chunk_size_bytes;                 /* SearchOptions.ChunkSizeBytes (0 = 1 000 000) */
} tsg_proto_request;
typedef struct tsg_proto_result {
  uint32_t n; /* TraceSearchMetadata, in object order */
  const uint8_t *trace_ids;     /* object ids (any length), trace_id_off / trace_id_len into this */
  const uint32_t *trace_id_off;
  const uint32_t *trace_id_len;
  const char *const *root_service_name; /* NUL-terminated, but proto strings may hold NUL bytes: */
  const char *const *root_trace_name;   /* read them with the lengths below */
  const uint64_t *start_time_unix_nano;
  const uint32_t *duration_ms;
  const uint32_t *object_idx;   /* position of the object in the block's iterator order */
  uint64_t inspected_traces, inspected_bytes, skipped_traces; /* SearchMetrics */
  uint64_t kernel_ns;
  const uint32_t *root_service_name_len;
  const uint32_t *root_trace_name_len;
} tsg_proto_result;
int tsg_proto_block_open(tsg_ctx *ctx, const char *block_dir, int device_hint, tsg_proto_block **out);
void tsg_proto_block_close(tsg_proto_block *b);
/* out[0] objects, out[1] pages (index records read), out[2] attribute keys, out[3] device bytes */
int tsg_proto_block_info(const tsg_proto_block *b, uint64_t out[4]);
/* TSG_E_CORRUPT (message in tsg_last_error) where Search returns an error: a trace that
 * fails to decode, an index/page/object framing error, reached before the limit break. */
int tsg_proto_search(tsg_ctx *ctx, tsg_proto_block *b, const tsg_proto_request *req, tsg_proto_result **out);
void tsg_proto_result_free(tsg_proto_result *r);

/* Go strconv semantics used by matchAttributes (tooling / tests): kind 0 ParseInt(s, 10, 64)
 * -> *i, 1 ParseFloat(s, 64) -> *f, 2 ParseBool -> *i. Returns 1 when Go returns err == nil. */
int tsg_go_parse(int kind, const char *s, size_t n, double *f, int64_t *i);

/* ---- block writer (tooling: synthetic data and test fixtures) ----------------- */
/* A v2 block from caller objects (ids ascending): data pages cut at
 * index_downsample_bytes (0 = 1 MiB), index, bloom, meta.json with the given page
 * encoding (0 none, 6 snappy) and dataEncoding ("v1" / "v2"). objs: concatenated object
 * bytes, obj_off: n + 1 offsets. */
int tsg_write_v2_block(const char *block_dir, const uint8_t (*ids)[16], const uint8_t *objs,
                       const uint64_t *obj_off, size_t n, int encoding, const char *data_encoding,
                       uint32_t index_downsample_bytes);
/* Entry list wire format (little endian), one record per trace:
 *   u32 id_len, id bytes, u64 start_ns, u64 end_ns, u32 ntags,
 *   ntags x (u32 klen, key, u32 vlen, value)
 * Restates NewBackendSearchBlock (tempodb/search/backend_search_block.go:28-129):
 * entries sorted ascending by id (duplicate ids rejected), tags lowercased,
 * one flatbuffer SearchPage per v2 data page cut when the builder bytes exceed
 * page_size_bytes, index pages of 100 KiB, header, search.meta.json.
 * encoding: backend.Encoding numeric value (0 none, 6 snappy). */
int tsg_write_search_block(const char *block_dir, const uint8_t *entries, size_t len,
                           int encoding, uint32_t page_size_bytes);

/* SearchEntryMutable.ToBytes (pkg/tempofb/search_entry_mutable.go:41-46) for one
 * entry in the wire format above; SearchBlockHeaderMutable.ToBytes from a list
 * of entries (pkg/tempofb/SearchBlockHeader_util.go:23-75). Free with tsg_free. */
/* StreamingSearchBlock.Append of each entry in order (one page per entry) into a search
 * WAL file; duplicates of an id stay separate pages (combined at replay). Test tooling. */
int tsg_write_wal_search(const char *path, const uint8_t *entries, size_t len, int encoding);
int tsg_fb_search_entry(const uint8_t *entry, size_t len, uint8_t **out, size_t *out_len);
int tsg_fb_search_header(const uint8_t *entries, size_t len, uint8_t **out, size_t *out_len);

/* Synthetic block generator (SURVEY.md §8 d): seeded, writes a search block with
 * n entries to block_dir. profile 0 = standard (~20 tags), 1 = high-cardinality
 * (adds long db.statement values). */
int tsg_synth_search_block(const char *block_dir, uint64_t n, uint64_t seed, int profile,
                           int encoding, uint32_t page_size_bytes);

/* Synthetic v2 trace block: n random 16-byte ids (returned sorted in ids_out if
 * non-NULL), dummy objects, bloom fp 0.01 / shard 100 KiB, index page 250 KiB,
 * data pages ~1 MiB (modules/storage/config.go:47-53). */
int tsg_synth_v2_block(const char *block_dir, uint64_t n, uint64_t seed, uint8_t (*ids_out)[16]);

#ifdef __cplusplus
}
#endif
#endif /* TSG_H */
