/*
 * libcep — MI355X-native complex-event-matching engine, C ABI.
 *
 * Drop-in boundary for the Siddhi runtime calls that flink-siddhi's
 * operator makes.  Every reference path below is relative to
 * core/src/main/java/org/apache/flink/streaming/siddhi/ in tammypi/flink-siddhi.
 * Plain C types only: pointers, sizes, status codes.  A JNI or Panama binding
 *  maps status codes onto the reference's exceptions.
 *
 * Threading: one cep_app per (Flink subtask, execution plan), as one
 * QueryRuntimeHandler per plan (operator/AbstractSiddhiOperator.java:114-176).
 * All calls come from one thread.  Matches are delivered through the output
 * callback on the calling thread, inside cep_flush(), before it returns —
 * the analogue of StreamCallback.receive(Event[]) running synchronously in
 * InputHandler.send (operator/StreamOutputHandler.java:63).
 *
 * Ownership: input buffers stay owned by the caller.  Host batches are
 * consumed before cep_send_batch() / cep_buffer_batch() return.  Device
 * batches (on_device = 1) are read asynchronously on the engine's HIP
 * stream: they must stay allocated and unchanged until that work is done —
 * after cep_flush(), or, for a caller whose allocator reuses memory in
 * stream order, after cep_stream_signal() has made the caller's stream wait
 * for the engine.  Output rows handed to the callback are owned by the engine
 * and valid only during the callback.  Snapshot buffers are engine-allocated
 * and released with cep_free().
 *
 * Hot-key probe: a keyed `every A -> B` runtime on the closed-form path
 * walks its first 2^20 rows as a short chunk and waits for it once inside
 * that cep_send_batch() (its hot-key verdict decides the next chunk's
 * routing); every later call returns without a sync.
 */
#ifndef CEP_H_
#define CEP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------
 * Mapping used by the Java shim:
 *   CEP_E_PARSE            -> SiddhiAppCreationException (fail-fast at DAG
 *                             build, AbstractSiddhiOperator.java:292-299)
 *   CEP_E_UNDEFINED_STREAM -> exception/UndefinedStreamException.java:20
 *                             (thrown at AbstractSiddhiOperator.java:205,
 *                              SiddhiOperatorContext.java:151)
 *   CEP_E_DUPLICATED_STREAM-> exception/DuplicatedStreamException.java:20
 *   CEP_E_UNSUPPORTED      -> valid SiddhiQL outside the engine subset
 *                             (joins, windows, tables): shim falls back to
 *                             real Siddhi
 *   CEP_E_ARG              -> IllegalArgumentException
 *                             (operator/StreamOutputHandler.java:89)
 *   CEP_E_DEVICE           -> HIP failure / no gfx950 device
 *   CEP_E_CAPACITY         -> per-key pending-state or key-space capacity
 *                             exceeded (raise cep_options.pending_slots /
 *                             pending_pool_log2 / key_capacity)
 *   CEP_E_STATE            -> snapshot incompatible with this plan
 */
enum {
  CEP_OK = 0,
  CEP_E_PARSE = 1,
  CEP_E_UNDEFINED_STREAM = 2,
  CEP_E_DUPLICATED_STREAM = 3,
  CEP_E_UNSUPPORTED = 4,
  CEP_E_ARG = 5,
  CEP_E_DEVICE = 6,
  CEP_E_CAPACITY = 7,
  CEP_E_STATE = 8
};

/* Attribute types: the Siddhi attribute types of utils/SiddhiTypeFactory.java:42-54
 * (STRING, INT, LONG, FLOAT, DOUBLE, BOOL; anything else OBJECT).
 * Column element layouts: INT int32, LONG int64, FLOAT float, DOUBLE double,
 * BOOL uint8 (0/1), STRING int32 dictionary id (cep_dict_intern). */
typedef enum {
  CEP_INT = 0, CEP_LONG = 1, CEP_FLOAT = 2, CEP_DOUBLE = 3, CEP_BOOL = 4,
  CEP_STRING = 5, CEP_OBJECT = 6
} cep_type;

typedef struct {
  char name[64];
  int32_t type;
} cep_attr;

typedef struct cep_options {
  int32_t device;          /* HIP device ordinal (default 0) */
  int32_t pending_slots;   /* per-key pending partial matches (default 16) */
  int64_t key_capacity;    /* partition / group keys are ints in [0, key_capacity) (default 1<<20) */
  int64_t chunk_events;    /* events per device chunk (default 1<<22) */
  int32_t buckets_log2;    /* key buckets per chunk, log2 (default 10) */
  int32_t profile;         /* k >= 1: time every k-th launch of each kernel with HIP events (cep_stats) */
  int32_t ordered_output;  /* 1: deliver matches in Siddhi's global emission
                              order; 0: per-key order (default 1) */
  int32_t key_stride;      /* multi-GPU: this shard owns keys with key % key_stride == key_offset (default 1/0) */
  int32_t key_offset;
  int32_t pending_pool_log2;  /* pending partials beyond pending_slots per key spill to a
                                 device pool of 2^n slots (default 20); closed-form
                                 patterns only, others fail with CEP_E_CAPACITY */
  int32_t sparse_keys;     /* 1: partition values are any int / long (a device hash map
                              assigns up to key_capacity dense slots; values come back
                              unchanged in `select s1.k`); 0: ints in [0, key_capacity) */
  int32_t late_policy;     /* event time (cep_watermark): a row older than rows an earlier
                              watermark released is a late event (counted in
                              cep_stats.late_events).  2: delivered, as the reference does
                              (default): it stays buffered and the next watermark releases it
                              with that watermark's rows in (ts, arrival) order, so the
                              engine sees a ts below ones it has processed
                              (AbstractSiddhiOperator.java:222-231 offers every row to the
                              PriorityQueue, :238-245 drains ts <= mark); `within` then
                              follows App. A.3's |ts(B) - ts(s1)| > W rule (ts_order 0; with
                              ts_order 1 a release holding late rows runs the order-tolerant
                              path against state kept in event-time form).
                              0: dropped; 1: dropped, and cep_watermark returns CEP_E_ARG
                              after releasing the on-time rows. */
  int32_t omit_seq;        /* 1: cep_rows.seq is NULL in callbacks and the seq column is not
                              copied to the host (StreamOutputHandler.receive,
                              operator/StreamOutputHandler.java:63-92, never reads it;
                              saves 8 B per delivered row); 0: delivered (default) */
  int32_t ts_order;        /* timestamps of the rows a pattern with `within` sees.
                              0 (default): any order, as the reference accepts (processing
                              time, late rows delivered by late_policy 2, any caller).  Such
                              patterns run the order-tolerant path: every row of the stream
                              a partial waits on is kept, and a partial is dropped exactly
                              when SURVEY App. A.3 drops it (|ts(event) - ts(s1)| > W, on
                              events of that stream), so the state and every match equal the
                              oracle's for any order.  `every A -> B` patterns take the
                              closed form's order-tolerant build (hot keys included; a
                              chunk's ts must lie within +-2^31 ms of its first row's, else
                              the flush fails with CEP_E_ARG), other shapes the N-state walk.
                              1: the caller guarantees non-decreasing ts (event-time order,
                              e.g. a watermark drain with late_policy 0): the event-time fast
                              paths (closed form, predicate push-down of B's, pruning at A
                              arrivals, hot keys), ~2x faster on config 3; a descent fails the
                              next cep_flush with CEP_E_ARG.  Sequences and multi-query groups
                              prune by |ts - ts(s1)| in any order either way (ts_order 1
                              only adds the check); the multi-GPU record / row shuffles
                              always run the event-time paths. */
  int32_t reserved[2];
} cep_options;

/* Fill *opt with defaults. */
void cep_default_options(cep_options* opt);

typedef struct cep_app cep_app;

/* A columnar batch of input events in arrival order.  `cols` follow the
 * attribute order of the stream definition (schema/StreamSchema.java:89-149,
 * the row order of schema/StreamSerializer.java:38-66).  A batch mixing
 * several input streams (per-row `stream` handles) requires identical
 * definitions for those streams. */
typedef struct {
  int64_t n;
  const int64_t* ts;          /* event timestamps, ms (InputHandler.send(ts, row)) */
  const uint8_t* stream;      /* per-row input handle, or NULL: all rows are `input` */
  int32_t input;              /* input handle (cep_input) when stream == NULL */
  int32_t ncols;
  const void* const* cols;    /* ncols column pointers */
  int32_t on_device;          /* 1: ts/stream/cols are device pointers */
} cep_batch;

/* Output rows, columnar, in emission order (see cep_options.ordered_output). */
typedef struct {
  const char* stream_id;
  int64_t n;
  int32_t ncols;
  const int64_t* ts;          /* output event timestamps (completing event) */
  const int64_t* seq;         /* arrival sequence number of the completing event */
  const void* const* cols;
} cep_rows;

typedef void (*cep_emit_fn)(void* user, const cep_rows* rows);

typedef struct {
  int64_t events_in;
  int64_t matches_out;
  int64_t batches;
  int64_t kernel_launches[16];
  double kernel_ms[16];       /* with cep_options.profile: summed HIP-event time */
  int64_t kernel_timed[16];   /* launches kernel_ms covers (profile = k: every k-th) */
  int64_t late_events;        /* rows dropped by cep_watermark as late (ts before an earlier release) */
  int64_t hot_keys;           /* closed-form path: keys matched by the hot-key kernels (hot.hip) */
} cep_stats_t;

/* Kernel kinds indexing cep_stats_t arrays. */
enum {
  CEP_K_FILTER = 0, CEP_K_PARTITION = 1, CEP_K_WALK = 2, CEP_K_ROUTE = 3,
  CEP_K_ORDER = 4, CEP_K_AGG = 5, CEP_K_OTHER = 6,
  CEP_K_CF_PARTITION = 7, CEP_K_CF_WALK = 8,  /* closed-form fast path (k_cfpart / k_cfwalk) */
  CEP_K_HOT = 9,                              /* hot-key matching (hot.hip, one entry per chunk) */
  CEP_K_MQ_PARTITION = 10, CEP_K_MQ_WALK = 11  /* multi-query groups (k_mqpart / k_mqwalk) */
};

/* ---- plan-level calls (no device needed) ------------------------------ */

/* SiddhiManager.validateSiddhiApp(plan)  — AbstractSiddhiOperator.java:295 */
int cep_validate(const char* plan, char* err, size_t errlen);

/* SiddhiTypeFactory.getStreamDefinition(plan, streamId) — utils/SiddhiTypeFactory.java:64-84
 * (the throw-away runtime used by returns(...) to infer output TypeInfo). */
int cep_plan_schema(const char* plan, const char* stream_id, cep_attr* out,
                    int cap, int* n, char* err, size_t errlen);

/* ---- runtime ----------------------------------------------------------- */

/* SiddhiManager.createSiddhiAppRuntime(plan) + start()
 * — AbstractSiddhiOperator.java:120-122,137-142.  NULL on error. */
cep_app* cep_create(const char* plan, const cep_options* opt, char* err,
                    size_t errlen);

/* SiddhiAppRuntime.shutdown() — AbstractSiddhiOperator.java:144-148 */
void cep_destroy(cep_app* app);

/* getStreamDefinitionMap().get(id) — AbstractSiddhiOperator.java:160-163 */
int cep_stream_schema(cep_app* app, const char* stream_id, cep_attr* out,
                      int cap, int* n);

/* getInputHandler(id) — AbstractSiddhiOperator.java:172.
 * Returns a handle >= 0, or -CEP_E_UNDEFINED_STREAM. */
int cep_input(cep_app* app, const char* stream_id);

/* addCallback(outId, StreamCallback) — AbstractSiddhiOperator.java:165-166 */
int cep_set_callback(cep_app* app, const char* out_id, cep_emit_fn fn,
                     void* user);

/* A batch of InputHandler.send(ts, row) calls — AbstractSiddhiOperator.java:130 */
int cep_send_batch(cep_app* app, const cep_batch* batch);

/* Event-time mode.  processElement — AbstractSiddhiOperator.java:222-231
 * (offer to the PriorityQueue<StreamRecord>): buffer rows in any timestamp
 * order on the device; nothing reaches the engine yet.  All rows buffered
 * between two watermarks share one input layout (`input`, stream column
 * present or not). */
int cep_buffer_batch(cep_app* app, const cep_batch* batch);

/* processWatermark(mark) — AbstractSiddhiOperator.java:238-247: the buffered
 * rows with ts <= mark go to the engine in (ts, arrival) order (one stable
 * device sort; the reference PQ orders by ts only, StreamRecordComparator.java:
 * 32-40); later rows stay buffered.  A row older than one already released
 * (a late event) is dropped and counted in cep_stats_t.late_events — `within`
 * needs event-time order; the reference would hand it to Siddhi out of order
 * — and the on-time rows of the same watermark are released as usual. */
int cep_watermark(cep_app* app, int64_t mark);

/* Rows still buffered (the PriorityQueue's size). */
int64_t cep_buffered(cep_app* app);

/* Deliver every match of the input sent so far to the callbacks; called
 * before emitWatermark / snapshotState / close (AbstractSiddhiOperator.java:246,331,316). */
int cep_flush(cep_app* app);

/* Device-resident consumers: expose the current (unflushed) output rows of
 * out_id as device pointers, valid until the next send/flush/reset. */
int cep_output_device(cep_app* app, const char* out_id, cep_rows* rows);

/* Drop unflushed outputs (device-resident consumers after reading them). */
int cep_reset_output(cep_app* app);

/* SiddhiAppRuntime.snapshot() — AbstractSiddhiOperator.java:374-380.
 * Restore is a TODO in the reference (AbstractSiddhiOperator.java:341);
 * cep_restore makes it real.  A snapshot restores only into a runtime of the
 * same compiled plan (plan hash and state geometry are checked; a mismatch is
 * CEP_E_STATE naming the cause).  Compatibility note (round 4): two-state
 * patterns whose s2 condition reads s1 compile to the N-state walk since
 * round 4, so their snapshots from earlier builds are refused unless the
 * restoring process sets CEP_PAIR_WALK=1 (the earlier two-state walk). */
int cep_snapshot(cep_app* app, uint8_t** buf, size_t* len);
int cep_restore(cep_app* app, const uint8_t* buf, size_t len);
void cep_free(void* p);

/* QueryRuntimeHandler.enable()/disable() — AbstractSiddhiOperator.java:150-156,
 * events sent while disabled are dropped (:128). */
int cep_set_enabled(cep_app* app, int enabled);

/* Device inputs produced on another HIP stream (a framework's current stream,
 * an RCCL collective): the engine's work queued after this call waits for
 * everything queued on hip_stream so far (event + stream wait, no host
 * sync).  Call before cep_send_batch / cep_route_batch / cep_send_records
 * with device pointers whose producer is still in flight. */
int cep_stream_wait(cep_app* app, void* hip_stream);

/* The reverse edge: everything queued on hip_stream after this call waits for
 * the engine's work queued so far (event + stream wait, no host sync).  A
 * framework that frees or reuses device input buffers in stream order (the
 * torch caching allocator) calls it after cep_send_batch / cep_route_batch /
 * cep_send_records so a recycled buffer is never overwritten while the
 * engine still reads it. */
int cep_stream_signal(cep_app* app, void* hip_stream);

/* String dictionary (STRING columns carry int32 ids). */
int32_t cep_dict_intern(cep_app* app, const char* s);
const char* cep_dict_lookup(cep_app* app, int32_t id);

int cep_stats(cep_app* app, cep_stats_t* out);
const char* cep_last_error(cep_app* app);

/* ---- multi-GPU key shuffle (Flink keyBy / router/DynamicPartitioner.java:43-60,
 * router/HashPartitioner.java:24-26) -------------------------------------
 * cep_route_batch evaluates the predicates of the app's (single) keyed
 * pattern over a device batch and writes the relevant events as fixed-size
 * records grouped by owner shard (key % world): records for shard r land in
 * rec_out[offsets[r] .. offsets[r]+counts[r]) in arrival order, offsets being
 * the exclusive prefix of counts_host.  seq0 = global arrival number of the
 * batch's first row (rank r of a job sends a contiguous global range).  A
 * record is cep_record_words(app) 8-byte words: [key | role<<32 | stream<<40,
 * seq, ts, carried columns...] (device memory, rec_out).  The caller
 * exchanges them (RCCL all-to-all) and feeds the received records, in
 * source-rank order, to the owner's app with cep_send_records. */
int cep_record_words(cep_app* app);               /* 8-byte words per record */
int cep_route_batch(cep_app* app, const cep_batch* batch, int world,
                    int64_t seq0, void* rec_out, int64_t rec_cap,
                    int64_t* counts_host);
int cep_send_records(cep_app* app, const void* recs, int64_t n,
                     int64_t events_represented);
/* Padded key shuffle: the step without a host round trip.  Like
 * cep_route_batch, but shard r's records land in a fixed segment of
 * 1 + seg_cap records at seg_out[r * (1 + seg_cap)]: one header record (word
 * 0 = the shard's record count | route error bits << 40 | 1 << 63 when the
 * count exceeds seg_cap; words 1 / 2 = seq / ts of the batch's first row),
 * then the records, then null records (role 0, seq / ts of the batch's last
 * row) up to seg_cap.  Nothing is read back: the call returns once the route
 * is queued on the engine's route stream.  The caller moves the segments with
 * one equal-split all-to-all (no host split sizes) and feeds the world
 * received segments, in source-rank order, to cep_send_records_padded, which
 * checks the headers on the device: a segment that overflowed seg_cap (its
 * excess records dropped) or carries a sender's route error makes the next
 * cep_flush / cep_watermark fail (CEP_E_CAPACITY / the route error).  That
 * step's output is then incomplete: like a failed Flink task, the caller
 * restores the last snapshot (cep_restore) and replays from it with the
 * two-phase exchange above or a larger seg_cap.  Needs a
 * non-empty batch (n > 0).  Replaces the same keyBy shuffle as
 * cep_route_batch (router/HashPartitioner.java:24-26). */
int cep_route_batch_padded(cep_app* app, const cep_batch* batch, int world,
                           int64_t seq0, void* seg_out, int64_t seg_out_cap,
                           int64_t seg_cap);
int cep_send_records_padded(cep_app* app, const void* segs, int world,
                            int64_t seg_cap, int64_t events_represented);
/* As cep_route_batch_padded, but an owner's records past seg_cap are not
 * lost: they go to spill_out (owner-grouped, each owner's in arrival order,
 * at most spill_cap records in all) and spill_counts[d] (a device array of
 * `world` int64, written asynchronously on the route stream) gets their
 * number.  Nothing is read back.  The caller learns about a spill when it
 * reads spill_counts (one step later, without stalling the pipeline); then,
 * instead of cep_send_records_padded, the owner concatenates per source rank
 * the segment's seg_cap records and that source's spilled records (shipped
 * in a second, exact exchange) and feeds them with cep_send_records: the
 * owner's input stays in global arrival order and no record is dropped
 * (flink_siddhi.shuffle.PaddedShuffle).  Only a spill past spill_cap fails
 * (CEP_E_CAPACITY at the next flush). */
int cep_route_batch_padded_spill(cep_app* app, const cep_batch* batch, int world,
                                 int64_t seq0, void* seg_out, int64_t seg_out_cap,
                                 int64_t seg_cap, void* spill_out, int64_t spill_cap,
                                 int64_t* spill_counts);
/* Make hip_stream wait for the routes queued so far (the route stream only:
 * the all-to-all of step s+1 need not wait for the walk of step s).  A host
 * batch's route runs on the engine stream and is joined into the route
 * stream, so this also covers it. */
int cep_route_signal(cep_app* app, void* hip_stream);
/* Row shuffle for apps with several queries (sequences, aggregations, more
 * than one pattern; BASELINE config 5 across GPUs).  No predicate push-down:
 * a sequence needs every row of its streams (strict contiguity).  Every row
 * some query reads is shipped whole as cep_row_words() int64 words
 * [stream handle, global arrival number, ts, one word per column] to owner
 * key % world, key = the stream's partition / group-by attribute (streams
 * only stateless filters read go round-robin by arrival number).  Rows come
 * out grouped by owner, in arrival order, like cep_route_batch; the owner
 * feeds what it received, in source-rank order, to cep_send_rows.
 * CEP_E_UNSUPPORTED when a stateful query is not keyed, or keys a stream on
 * two attributes, or the shipped streams differ in column types. */
int cep_row_words(cep_app* app);   /* < 0: -status */
int cep_route_rows(cep_app* app, const cep_batch* batch, int world, int64_t seq0, void* rec_out,
                   int64_t rec_cap, int64_t* counts_host);
int cep_send_rows(cep_app* app, const void* recs, int64_t n, int64_t events_represented);
/* Padded row shuffle: as cep_route_batch_padded, for whole rows.  Header and
 * null rows carry stream handle 31 (no input has it, so no query reads them):
 * header word 0 = 31 | route error bits << 8 | count << 32 | 1 << 63 on
 * overflow, words 1 / 2 = seq / ts of the batch's first row; null rows the
 * seq / ts of its last.  cep_send_rows_padded checks the headers on the
 * device and feeds the world segments (source-rank order) as one batch. */
int cep_route_rows_padded(cep_app* app, const cep_batch* batch, int world, int64_t seq0, void* seg_out,
                          int64_t seg_out_cap, int64_t seg_cap);
/* Whole rows with a spill, as cep_route_batch_padded_spill (received rows go
 * to cep_send_rows in the merged order). */
int cep_route_rows_padded_spill(cep_app* app, const cep_batch* batch, int world, int64_t seq0, void* seg_out,
                                int64_t seg_out_cap, int64_t seg_cap, void* spill_out, int64_t spill_cap,
                                int64_t* spill_counts);
int cep_send_rows_padded(cep_app* app, const void* segs, int world, int64_t seg_cap,
                         int64_t events_represented);

/* ---- dynamic plans (control events) ---------------------------------------
 * One operator hosting many plans, as AbstractSiddhiOperator keeps one
 * QueryRuntimeHandler per execution plan id (operator/AbstractSiddhiOperator.java:
 * 114-176) and changes the set on control events (onEventReceived, :400-467;
 * control/MetadataControlEvent.java, control/OperationControlEvent.java).
 * Plans are independent runtimes: changing one leaves the others' state. */
typedef struct cep_operator cep_operator;
cep_operator* cep_operator_create(const cep_options* opt, char* err, size_t errlen);
void cep_operator_destroy(cep_operator* op);
/* MetadataControlEvent: added / updated / deleted execution plans.  Update
 * replaces the plan's runtime (its state restarts, as the reference shuts
 * the old handler down); delete of an unknown id is ignored. */
int cep_operator_add_plan(cep_operator* op, const char* plan_id, const char* plan);
int cep_operator_update_plan(cep_operator* op, const char* plan_id, const char* plan);
int cep_operator_remove_plan(cep_operator* op, const char* plan_id);
/* OperationControlEvent ENABLE_QUERY / DISABLE_QUERY (query id = plan id). */
int cep_operator_enable(cep_operator* op, const char* plan_id, int enabled);
/* The plan's runtime (callbacks, stats, snapshot), or NULL. */
cep_app* cep_operator_plan(cep_operator* op, const char* plan_id);
/* A single-stream batch (batch->stream == NULL) of stream_id to every enabled
 * plan that reads it (router/AddRouteOperator.java:65-96); *plans_sent = plans
 * that took it.  A plan that fails does not stop the others: every plan gets
 * the batch, and the first failure (message prefixed with its plan id) is
 * returned after the loop. */
int cep_operator_send(cep_operator* op, const char* stream_id, const cep_batch* batch, int* plans_sent);
int cep_operator_flush(cep_operator* op);
/* Shared string dictionary of the operator's plans (STRING columns sent with
 * cep_operator_send carry these ids; a plan's output ids are the same). */
int32_t cep_operator_intern(cep_operator* op, const char* s);
const char* cep_operator_lookup(cep_operator* op, int32_t id);
/* Plan ids, newline separated. */
int cep_operator_plan_ids(cep_operator* op, char* buf, size_t len);
const char* cep_operator_last_error(cep_operator* op);

/* The input streams the plan's queries read (InputStream.getUniqueStreamIds
 * over its queries; the router's inputStreamToExecutionPlans,
 * router/AddRouteOperator.java:159-175), newline separated. */
int cep_plan_input_streams(const char* plan, char* buf, size_t len);
/* The plan's partition keys for stream_id: its queries' group-by attributes
 * (utils/SiddhiExecutionPlanner.java:76-140), newline separated. */
int cep_plan_partition_keys(const char* plan, const char* stream_id, char* buf, size_t len);
/* Dynamic-path routing of a device batch (router/AddRouteOperator.java:83-92,
 * router/DynamicPartitioner.java:43-60, router/HashPartitioner.java:24-26):
 * key = |Java hashCode(key_field)| (Integer, Long, Float, Double, Boolean,
 * String semantics), channel = key % nchan; key_field NULL / "" -> key -1 and
 * a pseudo-random channel.  chan_dev / keys_dev (optional): device arrays of
 * batch->n entries. */
int cep_partition_channels(cep_app* app, const cep_batch* batch, const char* key_field, int nchan,
                           int64_t seq0, int32_t* chan_dev, int64_t* keys_dev);

/* Synthetic workload generator (bench / tests only — BASELINE.md §3):
 * r(i,j) = splitmix64(seed ^ (i*0x9E3779B97F4A7C15) ^ j); key = r(i,0) mod K;
 * stream = r(i,1)>>63 (0 = A, 1 = B, or 0 when single_stream); id = r(i,2) mod 50;
 * price = (r(i,3)>>11) * 2^-53; ts = t0 + floor(i / rate).  Device pointers. */
int cep_generate(int64_t first, int64_t n, uint64_t seed, int64_t keys,
                 int64_t rate, int64_t t0, int single_stream, int32_t* key,
                 int64_t* ts, uint8_t* stream, int32_t* id, double* price,
                 void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* CEP_H_ */
