// Kernel argument blocks and launchers for the gfx950 kernels in kernels.hip.
// Host code (engine.cpp) fills these from a CompiledApp; everything is passed
// by value as kernel arguments (no per-launch allocation: graph-capturable).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "plan.h"

namespace cep {

// Columns of one input batch, in stream-definition order.
struct ColSet {
  const void* p[kMaxCols];
  int32_t t[kMaxCols];
  int32_t n;
};

// A contiguous slice [row0, row0 + n) of an input batch.
struct RowsArgs {
  ColSet cols;
  const int64_t* ts;
  const uint8_t* stream;   // per-row input handle, or nullptr
  int32_t input;           // handle when stream == nullptr
  int64_t row0;            // first row of the slice within the batch
  int64_t n;               // rows in the slice
  int64_t seq0;            // arrival sequence number of batch row 0
  int64_t prev_ts;         // ts of the row before the slice (monotonicity check)
  const int64_t* seq;      // per-row arrival numbers (rows received through the row
                           // shuffle, cep_send_rows), or nullptr: seq0 + row
  // Event-time order check (patterns with `within`, cep_options.ts_order =
  // 1): device word with the last ts of the previous batch (device batches:
  // the host does not see their ts), nullptr: none.
  const int64_t* prev_ts_dev;
};

__device__ __forceinline__ int64_t row_seq(const RowsArgs& r, int64_t row) {
  return r.seq ? r.seq[row] : r.seq0 + row;
}

struct VmArgs {
  const Ins* code;
  const uint64_t* konst;
};

// Output columns of one output stream (device).
struct OutArgs {
  void* col[kMaxOut];
  int32_t type[kMaxOut];
  int32_t prog[kMaxOut];   // program offset per output attribute
  int32_t src[kMaxOut];    // SRC_* direct source, or SRC_VM
  int32_t ncols;
  int64_t* ts;
  int64_t* seq;
  unsigned long long* count;   // rows written so far (atomic cursor)
  int64_t cap;
  int32_t write_seq;           // 0: nobody reads the arrival numbers (omit_seq, unordered output)
};

// Error flags (device word, OR-ed).
enum : uint32_t {
  ERR_KEY_RANGE = 1u,        // partition / group key outside [0, key_capacity)
  ERR_PENDING = 2u,          // per-key pending capacity exceeded
  ERR_ORDER = 4u,            // ts decreased inside a batch (within needs event-time order)
  ERR_OUT_CAP = 8u,          // output capacity exceeded (engine sizing bug)
  ERR_WINDOW = 16u,          // bucket window logic error
  ERR_POOL = 32u,            // pending overflow pool exhausted
  ERR_KEYMAP = 64u,          // more distinct partition values than key_capacity (sparse keys)
  ERR_TS_SPAN = 128u,        // a chunk's ts lie more than 2^31 ms either side of its first row
  ERR_SHUFFLE_CAP = 256u,    // padded key shuffle: an owner segment held more than seg_cap records
};

// Per-key state header: pending count (bits 0-7, <= S) | started << 8 |
// kHdrOvf: the list is longer than S and continues in the pending pool
// (closed-form path only; kext = count | pool run offset << 32).
constexpr uint32_t kHdrOvf = 1u << 9;

// ---------------------------------------------------------------- filter --
constexpr int kPref = 4;   // prefetched column slots of the fast paths

struct FilterArgs {
  RowsArgs rows;
  VmArgs vm;
  int32_t in_stream;
  int32_t filter_prog;     // -1: no filter
  TermList filter_terms;   // n >= 0: interpreter-free form of the filter
  OutArgs out;
  unsigned long long* tile_state;   // decoupled look-back words (zeroed per launch)
  unsigned int* ticket;             // tile ticket counter (zeroed per launch)
  unsigned int* err;
  // k_filterc (filter.hip): the predicate's distinct columns and each term's slot
  int32_t npref;
  int32_t pcol[kPref];
  int32_t fslot[kMaxTerms];
};

// ------------------------------------------------------- keyed pattern --
// `[every] s1=A[f] -> s2=B[g] [within W]` under `partition with`.
struct PatternArgs {
  int32_t a_stream, b_stream;
  int32_t f_prog;          // -1: true
  int32_t g_raw_prog;      // g evaluated in the partition pass (-1: true / in walk)
  TermList f_terms, g_terms;   // n >= 0: interpreter-free f / g_raw
  int32_t g_walk_prog;     // g evaluated per (pending, B) in the walk (-1: none)
  int32_t every;
  int64_t within;          // -1: none
  int32_t key_col_a, key_col_b;   // -1: unpartitioned (single key 0)
  int32_t nrec_a, nrec_b;
  int32_t rec_a[kMaxCaps], rec_b[kMaxCaps];   // columns carried in records
  int32_t ncap;                                // captured words per pending slot
  int32_t cap_from_rec[kMaxCaps];
  int32_t rec_words;       // 2 + max(nrec_a, nrec_b)
  int32_t slot_words;      // 2 + ncap
  int32_t key_words;       // per-key state block: 1 header word + S * slot_words
  int32_t pending_slots;   // S
  int64_t key_capacity;    // dense keys per shard
  int32_t key_stride, key_offset;   // shard ownership (key % stride == offset)
  int32_t buckets_log2;
  int32_t closed_form;     // 1: every && g independent of s1 -> data-parallel walk
  int32_t tolerant;        // 1: ts in any order (App. A.3 |ts(B) - ts(s1)| > W on every
                           // event of the waiting state's stream): keep every row of those
                           // streams, no pruning at A arrivals, no order check
  // group-by / having (agg_mode = 1): per-key running aggregates; state slot 0
  // holds (accumulator, count) word pairs per aggregate
  int32_t agg_mode;
  int32_t nagg;
  int32_t agg_fn[kMaxAggs];        // AGG_SUM / COUNT / AVG / MIN / MAX
  int32_t agg_arg_type[kMaxAggs];  // argument column type (record word as load_col)
  int32_t agg_out_type[kMaxAggs];
  int32_t agg_word[kMaxAggs];      // carried word of the argument (-1: count())
  int32_t having_prog;             // -1: none (LDCOL = carried word, LDAGG = running value)
  // N-state pattern / sequence (nfa_mode = 1): one NFA lane per key; a
  // partial is a state slot {start ts, state | count << 8, captures...}
  int32_t nfa_mode;
  int32_t nfa_pair;                // 1: a 2-state pattern's records and state layout (roles
                                   // A / B / G, slots {ts, -, s1 captures}) walked by the
                                   // N-state walk (order-tolerant runs: pool-backed lists)
  int32_t nfa_seq;                 // 1: sequence (strict contiguity, count states)
  int32_t nstates;
  int32_t stream_mask;             // input handles the query reads
  int32_t st_stream[kMaxStates];
  int32_t st_min[kMaxStates], st_max[kMaxStates];   // max -1: unbounded
  int32_t st_raw[kMaxStates];      // own-column condition (partition pass), -1: none
  int32_t st_walk[kMaxStates];     // condition reading captures (walk VM), -1: none
  int32_t st_tail_opt[kMaxStates]; // every state after j is optional (min 0)
  int32_t key_col_s[8];            // partition key column per input handle
  int32_t cap_state[kMaxCaps], cap_index[kMaxCaps], cap_word[kMaxCaps];
  uint64_t cap_null[kMaxCaps];      // a capture of a state that never matched: 0, or id -1 (null) for STRING
};

// Fast partition path: every column the pattern reads (key, f / g term
// columns, carried columns; at most kPref) is loaded for all of a lane's rows
// up front with 16-byte loads, so the tile's loads are in flight together.
constexpr int kPfRec = 2;        // carried words per record on the fast path
struct PrefPlan {
  int32_t n = -1;                // -1: generic path (per-use loads)
  int32_t col[kPref];
  int32_t f_slot[kMaxTerms], g_slot[kMaxTerms];
  int32_t key_slot = -1;         // -1: unkeyed
  int32_t reca_slot[8], recb_slot[8];
};

struct PartArgs {
  RowsArgs rows;
  PrefPlan pref;
  VmArgs vm;
  PatternArgs pat;
  int32_t from_records;        // 1: input rows are wide records (multi-GPU receive)
  const uint64_t* in_recs;     // wide records [hdr, seq, ts, carried...] when from_records
  int32_t in_rec_words;        // words per wide record
  int64_t* chunk_base;         // out: {ts, seq} of the chunk's first row (read by k_walk)
  int32_t tile_rows;           // rows per tile (2048)
  uint64_t* recs;              // out: records, tile-major
  uint16_t* tile_off;          // out: [ntiles][P+1] exclusive offsets
  uint64_t* stamps;            // diagnostics (CEP_STAMPS=1): per tile 16 s_memtime stamps
  unsigned int* err;
};

// Multi-GPU key shuffle (sender side).
constexpr int kMaxWorld = 64;

// Row shuffle for multi-query apps (cep_route_rows): every row a query reads
// is shipped whole as [stream, seq, ts, column words...] to owner key % world
// (key_col_s[stream] >= 0), or round-robin by arrival number for streams only
// stateless filters read (key_col_s = -1); key_col_s = -2: not shipped.
struct RowRouteArgs {
  RowsArgs rows;
  int32_t world;
  int32_t wrw;                 // 3 + columns
  int32_t tile_rows;
  int64_t seq0;                // global arrival number of batch row 0
  int32_t key_col_s[8];
  uint64_t* arena;             // [ntiles][tile_rows * wrw], owner-grouped per tile
  uint32_t* tcount;            // [ntiles][world]
  unsigned int* err;
  int64_t seg_cap;             // > 0: padded owner segments (cep_route_rows_padded)
  uint64_t* spill;             // see RouteArgs
  int64_t spill_cap;
  int64_t* spill_counts;
};

// Stream handle of the padded row shuffle's header and null rows: no input
// handle is ever this large (<= 8 streams), so no query reads them.
constexpr uint32_t kRowNullStream = 31;

struct RowUnpackArgs {
  const uint64_t* recs;
  int64_t n;
  int32_t wrw;
  int32_t ncols;
  void* col[kMaxCols];
  int32_t type[kMaxCols];
  int64_t* ts;
  uint8_t* stream;
  int64_t* seq;
};
struct RouteArgs {
  RowsArgs rows;
  VmArgs vm;
  PatternArgs pat;
  int32_t world;               // owners: key % world
  int32_t wrw;                 // wide record words: 3 + max(nrec_a, nrec_b)
  int32_t tile_rows;
  int64_t seq0;                // global arrival number of batch row 0
  uint64_t* arena;             // [ntiles][tile_rows * wrw], owner-grouped per tile
  uint32_t* tcount;            // [ntiles][world] kept rows per owner
  unsigned int* err;
  // > 0: padded segments (cep_route_batch_padded): owner d's records go to
  // out + (d * (1 + seg_cap) + 1) * wrw, at most seg_cap of them
  int64_t seg_cap;
  int32_t row_mode;            // padded segments of whole rows (cep_route_rows_padded)
  // padded with spill (cep_route_*_padded_spill): owner d's records past
  // seg_cap go to spill (owner-grouped, arrival order, at most spill_cap
  // records in all) and spill_counts[d] gets their number
  uint64_t* spill;
  int64_t spill_cap;
  int64_t* spill_counts;
};

struct WalkArgs {
  VmArgs vm;
  PatternArgs pat;
  const uint64_t* recs;
  const uint16_t* tile_off;
  int32_t ntiles;
  int32_t tile_rows;
  const int64_t* chunk_base;   // device {ts, seq} of the chunk's first row
  // per-key state, structure of arrays over the bucket-major key index
  // idx = bucket * keys_per_bucket + key_in_bucket (a bucket's keys are contiguous):
  //   khdr[idx]                    = pending count | started << 8
  //   kslot[(j * slot_words + w) * kstride + idx] = word w of pending slot j
  uint32_t* khdr;
  uint64_t* kslot;
  int64_t kstride;
  uint64_t* stamps;            // diagnostics (CEP_STAMPS=1): per block 16 s_memtime stamps
  OutArgs out;
  unsigned int* err;
  // N-state patterns / sequences: partial lists longer than pending_slots
  // (khdr bit kHdrOvf) keep slots [S, n) in a run of the pending pool, the
  // closed-form layout (kext = n | pool offset << 32, runs in pool_rd at
  // launch start; bit 31 of kext: the run is in pool_wr).  nullptr: no pool.
  uint64_t* kext;
  const uint64_t* pool_rd;
  uint64_t* pool_wr;
  unsigned long long* pool_cursor;
  uint64_t pool_cap;           // slots per pool
};

// ------------------------------------------ closed-form fast path (cf_kernels.hip) --
// `every s1=A[f] -> s2=B[g] within W` with f / g on the events' own columns,
// at most 2 physical carried words per record and plain-copy select items.
// Records are 8 + 8*nw bytes:
//   w0 = ts - chunk ts base (32) | row in tile (13) << 32 | role (3) << 45 | key in bucket (16) << 48
//   w1.. = physical carried words (A rows: A's, B rows: B's)
// A carried column whose buffer IS the event-ts buffer is not carried: its
// value is the record's ts (cap_phys / bcol_phys = -1).
#ifndef CF_TILE_ROWS
#define CF_TILE_ROWS 8192
#endif
constexpr int kCfItems = 8;                            // rows per lane
constexpr int kCfPartThreads = CF_TILE_ROWS / kCfItems;   // 512 (2 workgroups per CU) or 1024
constexpr int kCfTile = CF_TILE_ROWS;                  // rows per tile
constexpr int kCfWalkThreads = 512;
constexpr int kCfWindow = 2048;                        // records per LDS window (nw <= 1)
constexpr int kCfMaxKeys = 512;                        // keys per bucket
constexpr int kCfMaxTiles = (32 << 20) / kCfTile;      // chunk <= 32 Mi rows
constexpr int kCfMaxBuckets = 4096;
constexpr int kCfMaxCaps = 2;                          // captured words per pending slot
constexpr int kCfMaxOut = 8;                           // select items on the fast path

struct CfPlan {
  int32_t nw;                      // physical carried words per record (0..2)
  int32_t a_slot[2], b_slot[2];    // prefetch slot of physical word w (A rows / B rows)
  int32_t a_log[2], b_log[2];      // received records: logical carried word of physical word w
  int32_t cap_phys[kMaxCaps];      // A capture i -> physical word, -1 = the A's event ts
  int32_t bcol_phys[kMaxCaps];     // B record word c (SRC_REC + c) -> physical word, -1 = ts
};

// Hot keys (hot.hip): keys whose records would make their bucket a straggler
// (Zipf-skewed streams) are diverted by k_cfpart into hot buckets P + h
// (h < kCfHotMax, one per key) and matched by grid-wide scans instead of one
// workgroup per bucket.
constexpr int kCfHotMax = 1024;
constexpr int kHotBlock = 2048;                     // hot records per scan block
constexpr uint16_t kNotHot = 0xffff;

struct CfPartArgs {
  RowsArgs rows;
  const uint16_t* hot_id;      // dense key -> hot slot (kNotHot), nullptr: no diversion
  int32_t nhot;                // hot buckets after the P key buckets (0 or kCfHotMax)
  PrefPlan pref;
  int32_t ts_slot;             // prefetch slot whose column IS the event-ts buffer (-1: none)
  // received shuffle records (cep_send_records): rows are wide records
  // [hdr = key | role << 32 | stream << 40, global seq, ts, logical carried...]
  const uint64_t* in_recs;     // nullptr: rows are columns
  int32_t in_rec_words;
  PatternArgs pat;
  CfPlan cf;
  int64_t* chunk_base;         // out: {ts, seq} of the chunk's first row
  uint64_t* recs;              // out: records, tile t at recs + t * kCfTile * (1 + nw)
  uint16_t* tile_off;          // out: [P+1][ntiles] exclusive bucket offsets, bucket-major
  int32_t ntiles;
  uint64_t* stamps;            // diagnostics (CEP_STAMPS=1): per tile 16 s_memtime stamps
  unsigned int* err;
};

struct CfWalkArgs {
  PatternArgs pat;
  CfPlan cf;
  const uint64_t* recs;
  const uint16_t* tile_off;
  int32_t ntiles;
  const int64_t* chunk_base;
  uint32_t* khdr;              // per-key state, same layout as WalkArgs
  uint64_t* kslot;
  int64_t kstride;
  uint64_t* kext;              // per key: count | overflow run offset << 32 (header bit kHdrOvf)
  const uint64_t* pool_rd;     // pending pool this launch reads overflow runs from
  uint64_t* pool_wr;           // ... and writes rebuilt runs to (slot s word w at [s * slot_words + w])
  unsigned long long* pool_cursor;   // slots allocated in pool_wr (zeroed per launch)
  uint64_t pool_cap;           // slots per pool
  const uint64_t* key_rev;     // sparse keys: dense key -> partition value (nullptr: dense keys)
  const uint16_t* hot_id;      // diversion active: hot keys are not this launch's (nullptr: none)
  uint64_t* hot_cand;          // records << 32 | dense key of keys over hot_thresh this launch
  uint32_t* hot_ncand;
  uint32_t hot_thresh;         // 0: no candidate collection
  OutArgs out;
  const uint64_t* in_seq;      // received records: &record[row0].seq (global arrival numbers), else nullptr
  int32_t in_rec_words;
  uint64_t* stamps;
  int32_t ablate;              // diagnostics (CEP_ABLATE): bit 0 no emission, 1 no commit, 2 no rank/reload
  unsigned int* err;
};

struct HotArgs {
  PatternArgs pat;
  CfPlan cf;
  const uint64_t* recs;        // k_cfpart records (tile-major)
  const uint16_t* tile_off;    // [P + kCfHotMax + 1][ntiles]
  int32_t ntiles;
  const int64_t* chunk_base;
  uint16_t* hot_id;            // [key_capacity] dense key -> slot
  int32_t* hot_key;            // [kCfHotMax] slot -> dense key (-1: free)
  uint32_t* hot_m;             // [kCfHotMax] records this chunk
  uint32_t* hot_gbase;         // [kCfHotMax + 1] exclusive prefix of hot_m (last: M)
  uint32_t* hoff;              // [kCfHotMax][ntiles] a slot's records before tile t
  uint64_t* cand;              // walk candidates: records << 32 | dense key
  uint32_t* ncand;
  uint32_t cand_cap;
  uint32_t thresh;
  uint64_t* harr;              // hot records, grouped by slot, arrival order
  uint32_t* hrow;              // chunk-relative row of each hot record
  uint32_t* hnb;               // next B of the slot after each record (kNoPos: none)
  uint32_t* bsum;              // per block: first slot, first B of it (incl.), last slot, carry
  uint32_t* bcnt;              // per block: record matches
  uint32_t* boff;
  uint32_t* hcm;               // per slot: carried partials completed, first completed index
  // order-tolerant builds (pat.tolerant): per hot record the ts range
  // [htmn, htmx] (record ts units) of the B-stream rows from it to its slot's
  // next g-passing B inclusive (empty: htmn > htmx); hflag bit 0 = that range
  // still open at the block end, bit 1 = an A that survives to its next B /
  // the slot end; per block its first record's range [mn, mx, open] (btol)
  uint32_t* htmn;
  uint32_t* htmx;
  uint8_t* hflag;
  uint32_t* btol;
  unsigned long long* obase;   // [0]: output base, [1]: carried rows total
  int32_t max_blocks;
  uint32_t* khdr;
  uint64_t* kslot;
  int64_t kstride;
  uint64_t* kext;
  const uint64_t* pool_rd;
  uint64_t* pool_wr;
  unsigned long long* pool_cursor;
  uint64_t pool_cap;
  const uint64_t* key_rev;
  OutArgs out;
  uint32_t* active;            // out: slots in use after the update
  const uint64_t* in_seq;      // received shuffle records: &record[row0].seq, else nullptr
  int32_t in_rec_words;
  int32_t ablate;              // diagnostics (CEP_HOT_ABLATE, wrong results): 1 no gather sort, 2 no gather copy
  unsigned int* err;
};

// Fast route (k_cfroute): the k_cfpart load path for the sender side of the
// key shuffle (8192-row tiles, prefetched columns, term-list f / g).
struct CfRouteArgs {
  RouteArgs r;                 // r.tile_rows = kCfTile
  PrefPlan pref;
  int32_t ts_slot;             // prefetch slot whose column IS the event-ts buffer (-1: none)
};

// Sparse partition keys (keymap.hip): value -> dense key slot.
struct KeyMapArgs {
  const void* key;             // key column (int32 or int64), batch rows
  int32_t key_is_long;
  const uint8_t* stream;       // per-row input handle or nullptr
  int32_t input, a_stream, b_stream;
  int64_t row0, n;
  unsigned long long* tkey;    // table: stored value + 1 (0 = empty)
  uint32_t* tval;              // table: dense id
  uint64_t table_cap;          // power of two
  uint64_t* rev;               // dense id -> value
  unsigned int* count;         // dense ids handed out
  unsigned int* minus_one;     // dense id of the value -1 (0xffffffff: none yet)
  uint32_t cap;                // key_capacity
  int32_t* out;                // dense id per row (row i of the slice)
  unsigned int* err;
};

// Dynamic-path routing key per row (keymap.hip).
struct RouteKeyArgs {
  const void* col;             // key field column (nullptr: no group-by key -> random channel)
  int32_t type;
  int64_t n;
  const int32_t* str_hash;     // STRING: Java String.hashCode() per dictionary id
  int32_t nstr;
  int32_t nchan;
  int64_t seq0;                // arrival number of row 0 (random channel draw)
  int64_t* keys;               // out: partition key (-1: none), or nullptr
  int32_t* chan;               // out: channel
};

// -------------------------------- multi-query groups (mq_kernels.hip) --
// One app's keyed queries that share a partition / group-by key column and
// whose per-event work is interpreter-free (sequences of the one-live-partial
// shape, group-by aggregations), processed together: ONE partition pass over
// the batch evaluates every query's conditions into a per-record bit mask
// (conditions deduplicated per input stream), ONE walk per key bucket runs
// all the queries over each key's records (lane = key, wave = query).
// Records are 16 + 8 * nc bytes:
//   w0 = ts - chunk ts base (32) | row in chunk (25) << 32 | stream (3) << 57
//   w1 = condition bits of the row's stream (47) | always-true bit 47 | key in bucket (16) << 48
//   w2.. = physical carried columns
constexpr int kMqMaxQ = 64;            // queries per group
constexpr int kMqMaxCond = 47;         // distinct conditions per input stream
constexpr int kMqTrueBit = 47;         // record bit that is always set (condition-free states)
constexpr int kMqMaxCarry = 4;         // logical carried columns per group
constexpr int kMqMaxPhys = 4;          // physical carried words per record
constexpr int kMqMaxCaps = 4;          // captures per sequence
constexpr int kMqMaxSel = 8;           // select items per query
constexpr int kMqMaxAggs = 4;
constexpr int kMqTile = 16384;         // rows per partition tile (1024 lanes x 16)
constexpr int kMqPartThreads = 1024;
constexpr int kMqWalkThreads = 1024;   // 16 waves; one workgroup per CU
constexpr int kMqWindow = 4096;        // records per walk window (LDS)
constexpr int kMqMaxTiles = (16 << 20) / kMqTile;   // chunk <= 16 Mi rows
constexpr int kMqMaxKpb = 1024;        // keys per bucket
constexpr int kMqMaxBuckets = 8192;
// Records per k_mqwalk LDS window by physical carried words: what fits beside
// the per-wave row staging (kMqStgWords) under 160 KB of LDS.
constexpr int mq_window(int nc) { return nc <= 0 ? 4096 : nc == 1 ? 3072 : nc <= 3 ? 2048 : 1536; }
constexpr int kMqStgWords = 320;       // per wave: staged output rows (column-major)
enum : int32_t { MQ_SEQ = 0, MQ_AGG = 1 };
enum : int32_t { MQ_SRC_KEY = 14, MQ_SRC_TS = 15 };   // capture / carried sources beside words 0..3

struct MqCond {                   // one distinct condition of one input stream
  TermList tl;
  int32_t slot[kMaxTerms];        // prefetched column slot of each term
};

// Per-query descriptor (device array; read with wave-uniform indices).
struct MqQuery {
  int32_t kind;                   // MQ_SEQ / MQ_AGG
  int32_t nwords;                 // state words per key
  int64_t st_off;                 // first state word (state + st_off * kstride + w * kstride + key idx)
  // sequence: states packed per field (state j at bits j * width)
  int32_t nstates, every;
  int64_t within;                 // -1: none
  uint32_t stream_mask;           // input handles the query reads
  uint32_t st_stream;             // 3 bits per state
  uint64_t st_bit;                // 6 bits per state: record condition bit
  uint64_t st_min, st_max;        // 8 bits per state; max 255 = unbounded
  uint32_t tail_opt;              // bit j: every state after j is optional
  int32_t ncap;
  int32_t cap_state[kMqMaxCaps], cap_last[kMqMaxCaps], cap_src[kMqMaxCaps];   // src: logical word / MQ_SRC_*
  // aggregation
  int32_t in_stream, filter_bit, nagg;
  int32_t agg_fn[kMqMaxAggs], agg_arg_type[kMqMaxAggs], agg_out_type[kMqMaxAggs], agg_src[kMqMaxAggs];
  int32_t hav_item, hav_cop, hav_ctype;   // hav_item -1: no having
  uint64_t hav_cconst;
  // select items: SRC_KEY, SRC_CAP + i (sequence), SRC_AGG + i, SRC_REC + logical word (aggregation);
  // sel_vi: the item's slot in the walk's row value array (0 key, 1 + i capture / aggregate i,
  // 5 + w logical carried word w), sel_w: its column width in bytes
  int32_t nsel;
  int32_t sel_src[kMqMaxSel], sel_type[kMqMaxSel], sel_vi[kMqMaxSel], sel_w[kMqMaxSel];
  int32_t hav_vi;                 // having item's value slot
  // output stream (rewritten when the engine grows it)
  void* out_col[kMqMaxSel];
  int64_t* out_ts;
  int64_t* out_seq;
  unsigned long long* out_count;
  int64_t out_cap;
};

// Walk units: what one wave runs over a block of 64 keys.
//   MQU_SEQ     one sequence query (general shape, its own partial per key);
//   MQU_SEQ_BP  a class of sequence queries of one shape whose states read
//               distinct streams and count at most "one or more": all of a
//               key's live partials then share state, start and captures, so
//               the class advances bit-parallel (a live mask per key, one bit
//               per query; the per-state conditions of the class are a run of
//               consecutive record bits in query order);
//   MQU_AGG     up to 8 aggregations of one shape (stream, functions,
//               arguments, select / having layout), each query's running
//               values in the lane's registers: the record is decoded once.
enum : int32_t { MQU_SEQ = 0, MQU_SEQ_BP = 1, MQU_AGG = 2 };
struct MqUnit {
  int32_t kind;
  int32_t q0, nq;                 // descriptors [q0, q0 + nq)
  int32_t nu;                     // MQU_AGG: queries held in registers (template width)
  int32_t fast;                   // MQU_AGG: mq_agg_fast shape (0: generic mq_agg_unit; 1 sum / avg double,
                                  // 2 sum long, 9 count only)
  // MQU_SEQ_BP: class state words at st_off (live mask, started mask, state, start ts, captures)
  int64_t st_off;
  uint32_t st_of_stream;          // 4 bits per input handle: state + 1 (0: the class does not read it)
  uint64_t allow;                 // bit j * 8 + s: a partial in state j moves to (or stays in) state s
  uint64_t cbase;                 // 8 bits per state: first record bit of the class's condition run (0xff: none)
  uint32_t keep_last;             // the last state collects more (unbounded) after emitting
};

struct MqPartArgs {
  RowsArgs rows;
  PrefPlan pref;                  // prefetched columns: key, condition columns, carried columns
  int32_t ts_slot;                // slot whose column IS the event-ts buffer (-1: none)
  uint32_t stream_mask;           // input handles some group query reads
  int32_t key_slot;               // slot of the key column
  int32_t ncond[8];               // conditions per input handle
  const MqCond* conds;            // [8][kMqMaxCond]
  int32_t nphys;                  // physical carried words
  int32_t phys_slot[kMqMaxPhys];  // slot of physical carried word w
  int32_t check_order;            // 1: some query has `within` (ts order check)
  int64_t key_capacity;
  int32_t key_stride, key_offset;
  int32_t buckets_log2;
  int32_t ntiles;
  int64_t* chunk_base;            // out: {ts, seq} of the chunk's first row
  uint64_t* recs;                 // out: tile t at recs + t * kMqTile * (2 + nphys)
  uint16_t* tile_off;             // out: [P + 1][ntiles] bucket-major exclusive offsets
  unsigned int* err;
};

struct MqWalkArgs {
  const MqQuery* q;
  int32_t nq;
  const MqUnit* units;
  int32_t nunits;
  int32_t nphys;
  int32_t lmap[kMqMaxCarry];      // logical carried word -> physical word, -1: the event ts
  const uint64_t* recs;
  const uint16_t* tile_off;
  int32_t ntiles;
  int32_t buckets_log2;
  int32_t kpb;                    // keys per bucket
  int32_t key_stride, key_offset;
  const int64_t* chunk_base;
  const int64_t* in_seq;          // per-row arrival numbers of the chunk (row shuffle), or nullptr
  uint64_t* state;                // per bucket, per state word, the bucket's kpb keys: bucket b's state
                                  // is one contiguous block of words * kpb (few pages per workgroup)
  int64_t kstride;
  int64_t words;                  // state words per key
  uint64_t* stamps;               // diagnostics (CEP_STAMPS=1): per bucket 16 s_memtime stamps
  int32_t ablate;                 // diagnostics (CEP_MQ_ABLATE): 1 = rows counted, not stored
  unsigned int* err;
};

// --------------------------------------------------------------- launchers --
void launch_mq_partition(const MqPartArgs& a, hipStream_t s);
void launch_mq_walk(const MqWalkArgs& a, int nbuckets, hipStream_t s);
void launch_cf_partition(const CfPartArgs& a, int64_t ntiles, hipStream_t s);
void launch_cf_walk(const CfWalkArgs& a, int nbuckets, hipStream_t s);
void launch_keymap(const KeyMapArgs& a, hipStream_t s);
void launch_route_keys(const RouteKeyArgs& a, hipStream_t s);
void launch_hot_match(const HotArgs& a, hipStream_t s);
void launch_hot_update(const HotArgs& a, int diverted, hipStream_t s);
void launch_filter(const FilterArgs& a, int64_t ntiles, bool vm, hipStream_t s);
// coalesced compaction filter (filter.hip): term-list predicate over <= 3
// columns, plain projection; rows per tile
void launch_filterc(const FilterArgs& a, int64_t ntiles, hipStream_t s);
int filterc_rows_per_tile();
void launch_partition(const PartArgs& a, int64_t ntiles, bool vm, hipStream_t s);
void launch_route(const RouteArgs& a, int64_t ntiles, bool vm, uint32_t* toffs,
                  unsigned long long* dcount, uint64_t* out, hipStream_t s);
void launch_route_collect(const RouteArgs& a, int64_t ntiles, uint32_t* toffs,
                          unsigned long long* dcount, uint64_t* out, hipStream_t s);
// padded key shuffle: segment headers + null tails (sender), header check (owner)
void launch_route_pad(const RouteArgs& a, const unsigned long long* dcount, uint64_t* out, hipStream_t s);
void launch_route_check(const uint64_t* segs, int world, int64_t seg_cap, int wrw, int row_mode, unsigned int* err,
                        hipStream_t s);
void launch_route_rows(const RowRouteArgs& a, int64_t ntiles, uint32_t* toffs,
                       unsigned long long* dcount, uint64_t* out, hipStream_t s);
void launch_unpack_rows(const RowUnpackArgs& a, hipStream_t s);
void launch_cf_route(const CfRouteArgs& a, int64_t ntiles, hipStream_t s);
void launch_walk(const WalkArgs& a, int nbuckets, bool vm, hipStream_t s);
// event-time reorder (reorder.hip)
size_t reorder_temp_bytes(int64_t n);
int reorder_sort(void* temp, size_t temp_bytes, const int64_t* keys_in, int64_t* keys_out, int32_t* idx_in,
                 int32_t* idx_out, int64_t n, hipStream_t s);
void launch_upper_bound(const int64_t* sorted, int64_t n, int64_t wm, int64_t* out3, hipStream_t s);
void launch_gather(const void* src, void* dst, const int32_t* perm, int64_t first, int64_t n, int width,
                   hipStream_t s);
// output emission order (reorder.hip): seq range / descents, stable seq sort
void launch_seq_stats(const int64_t* seq, const unsigned long long* count, int64_t cap, unsigned long long* out3,
                      hipStream_t s);
size_t order_temp_bytes(int64_t n);
int order_sort(void* temp, size_t temp_bytes, const int64_t* seq, int64_t n, int64_t lo, int bits, void* keys_a,
               void* keys_b, int32_t* idx_a, int32_t* idx_b, hipStream_t s);
void launch_generate(int64_t first, int64_t n, uint64_t seed, int64_t keys,
                     int64_t rate, int64_t t0, int single_stream, int32_t* key,
                     int64_t* ts, uint8_t* stream, int32_t* id, double* price,
                     hipStream_t s);

// 512 lanes x 16 rows: 8192-row tiles halve the decoupled look-back chains
// of 4096-row tiles (config 2: 907 -> 830 us per 10^8 events)
constexpr int kFilterThreads = 512;   // 1024 lanes (16384-row tiles): 878 us
constexpr int kFilterItems = 16;          // rows per thread per tile
constexpr int kPartThreads = 512;
constexpr int kPartItems = 4;             // tile = 2048 rows
constexpr int kWalkThreads = 512;
constexpr int kWalkWindow = 1024;         // records per LDS window
constexpr int kWalkMaxTiles = 8192;       // tiles per chunk (16 Mi rows)
constexpr int kWalkMaxKeys = 512;         // keys per bucket (LDS histogram)
constexpr int kWalkCapLds = 2;            // carried record words kept in LDS (closed form)
constexpr int kMaxPending = 16;           // pending_slots upper bound (walk LDS lists)

}  // namespace cep
