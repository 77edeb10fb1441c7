// api.hip — the C-ABI of libdeltagpu (include/deltagpu.h): engine lifecycle,
// argument validation, scratch management and kernel sequencing.  Errors follow
// the header's conventions; nothing here falls back to a CPU path.
#include <mutex>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/deltagpu.h"
#include "dg_hash.h"
#include "dg_launch.h"

using namespace dg;

struct dg_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // decoupled look-back scratch
  u64* state = nullptr;
  u64 state_cap = 0;
  u32* ticket = nullptr;  // [0] ticket, [1] error bits, [2] store_check flag, [3] op order flag,
                          // [4] join abort epoch, [6] the Merkle build/update arrival counter
                          // (16 words right behind d_counts: one allocation, see below)
  u32* counts = nullptr;  // single-pass join tile-count granules
  u32* started = nullptr;  // single-pass join start flags (JOIN_MAX_GRID epochs)
  u64 counts_cap = 0;
  // ping-pong intermediate states of dg_joink / dg_apply_deltas
  void* fold = nullptr;
  size_t fold_cap = 0;
  bool splice = true;  // sparse keyed joins as a splice (DG_SPLICE=0: the full join)
  // the splice's taken rows, edit and per-key index (its own: a stepwise fold's joins
  // splice while their inputs live in `fold`)
  void* spl = nullptr;
  size_t spl_cap = 0;
  // dg_join_delta's union context on its full-join path (its own: the join it calls may
  // splice through `spl`)
  void* ubuf = nullptr;
  size_t ubuf_cap = 0;
  // dg_join_delta_home's scratch: the edit, the per-key index, the result header
  void* sml = nullptr;
  size_t sml_cap = 0;
  // dg_join_delta's one-wait path (kdelta.hip): per-key figures, the splice index, the
  // union context (DG_KD=0: the splice path with its host waits, for A/B)
  void* kdb = nullptr;
  size_t kdb_cap = 0;
  void* kdz = nullptr;  // its tree update's dirty flags and chunk row-count changes: zero
  size_t kdz_cap = 0;   //   between calls (the re-reduction consumes them)
  bool kd = true;
  // the full diff's per-group key sums: two buffers of diff_bsum_cap words, zero when
  // allocated; a call adds into one and its write kernel zeroes the other, which the
  // previous call used (no memset launch per diff)
  u64* diff_bsum = nullptr;
  u64 diff_bsum_cap = 0;
  int diff_parity = 0;
  u32 epoch = 0;
  // small device counters + pinned host mirror.  d_counts[0..8) and ticket[0..16) are one
  // device allocation (ticket == (u32*)(d_counts + 8)), so a synchronous call brings its
  // counts and the error bits home in ONE copy (read_counts).
  u64* d_counts = nullptr;  // 8 entries, then the ticket words
  u64* h_counts = nullptr;  // pinned, 16 entries (a mirror of the whole block)
  // synchronous calls: a one-wave kernel copies the counts into host-coherent mapped memory
  // and then stores a sequence number there, which the host polls (read_counts)
  u64* h_pub = nullptr;  // mapped host memory, 24 words: [0..16) the block, [16] the sequence
  u64* d_pub = nullptr;  // its device address
  u64 pub_seq = 0;
  u32 h_ticket[16] = {};  // the ticket words as of the last synchronous call
  u32 last_err_bits = 0;  // the error bits read_counts last failed on (0: it did not)
  // general scratch
  void* tmp = nullptr;
  size_t tmp_cap = 0;
  int join_mode = JOIN_SINGLE_PASS;  // DG_JOIN_MODE=2: two-pass count/compact variant
  int join_workers = 0;           // persistent pass-1 workgroups (0: all resident ones)
  // dg_apply_deltas: 0 one pass per <= 64 deltas, delta by delta where an input needs it;
  // DG_APPLY_MODE=fold: always delta by delta; =onepass: never (DG_E_INVAL instead)
  int apply_mode = 0;
  void* h_stage = nullptr;        // pinned staging of kernel descriptors
  size_t h_stage_cap = 0;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;  // hand-offs to the device's shared join stream
  // asynchronous calls since the last dg_engine_sync, replayed there (joins on the
  // two-pass kernels) when a single-pass join grid aborted for lack of residency
  struct Pending {
    int kind;  // 0 dg_join2_async, 1 dg_merkle_build_async
    dg_store a, b, out;
    dg_context ca, cb, out_ctx;
    const uint64_t* keys;
    uint64_t n_keys;
    uint64_t* d_counts;
    dg_merkle t;
    dg_merkle* tp;
  };
  std::vector<Pending> pending;
};

// The single-pass join kernel is persistent: its workgroups wait on each other, so two
// of its grids must never be in flight on one device at once (each could hold CUs the
// other's waiting workgroups need).  While a device has one engine, its joins run on
// the engine's stream.  With several, every engine's join kernels run on one shared
// stream per device, ordered with the engine's own stream by events
// (tests/test_gpu_concurrency.py).  Against other streams' and processes' kernels the
// grid checks its own residency and aborts (join.hip, stripe_sums); the calls then re-run
// on kernels that do not wait (dg_join2, dg_engine_sync, dg_join2_changes).
struct DevShare {
  int engines = 0;
  hipStream_t stream = nullptr;
};
std::mutex g_share_mu;
DevShare g_share[64];

// The device's shared join stream, or nullptr while e is the only engine on its device.
hipStream_t shared_join_stream(dg_engine* e) {
  std::lock_guard<std::mutex> g(g_share_mu);
  DevShare& d = g_share[e->device & 63];
  if (d.engines < 2) return nullptr;
  if (!d.stream && hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess)
    d.stream = nullptr;
  return d.stream;
}

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return fail(DG_E_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                  __FILE__, __LINE__);                                                   \
  } while (0)

int set_device(dg_engine* e) {
  HIP_TRY(hipSetDevice(e->device));
  return DG_OK;
}

int ensure_state(dg_engine* e, u64 tiles) {
  if (tiles <= e->state_cap) return DG_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->state) HIP_TRY(hipFree(e->state));
  e->state = nullptr;
  u64 cap = std::max<u64>(tiles, 1024);
  if (hipMalloc(&e->state, cap * sizeof(u64)) != hipSuccess)
    return fail(DG_E_NOMEM, "hipMalloc of %llu look-back granules failed", cap);
  // zeroed ON the engine stream: a plain hipMemset runs on the null stream, which is not
  // ordered with a non-blocking engine stream, and could land after the next kernel
  // has already written this array
  HIP_TRY(hipMemsetAsync(e->state, 0, cap * sizeof(u64), e->stream));
  e->state_cap = cap;
  // the epoch stays monotonic: the tile-count granules (e->counts) outlive this array,
  // and a restarted epoch would make their stale values read as current
  return DG_OK;
}

int ensure_tmp(dg_engine* e, size_t bytes) {
  if (bytes <= e->tmp_cap) return DG_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->tmp) HIP_TRY(hipFree(e->tmp));
  e->tmp = nullptr;
  size_t cap = std::max<size_t>(bytes, 1 << 20);
  if (hipMalloc(&e->tmp, cap) != hipSuccess)
    return fail(DG_E_NOMEM, "hipMalloc of %zu scratch bytes failed", cap);
  e->tmp_cap = cap;
  return DG_OK;
}

// the full diff's two group-sum buffers (see dg_engine::diff_bsum), grown on demand
int ensure_diff_bsum(dg_engine* e, u64 groups) {
  if (groups <= e->diff_bsum_cap) return DG_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->diff_bsum) HIP_TRY(hipFree(e->diff_bsum));
  e->diff_bsum = nullptr;
  e->diff_bsum_cap = 0;
  if (hipMalloc(&e->diff_bsum, 2 * groups * sizeof(u64)) != hipSuccess)
    return fail(DG_E_NOMEM, "hipMalloc of %llu diff group sums failed", (unsigned long long)groups);
  HIP_TRY(hipMemsetAsync(e->diff_bsum, 0, 2 * groups * sizeof(u64), e->stream));
  e->diff_bsum_cap = groups;
  return DG_OK;
}

Rows rows_of(const dg_store* s);
MerkleT merkle_of(const dg_merkle* t);

// one full diff enqueued: the group sums of this call and the ones its write kernel zeroes
// (all g words: a call of another depth may have dirtied more groups than this one has)
hipError_t enqueue_merkle_diff(dg_engine* e, const dg_merkle* a, const dg_store* sa, const dg_merkle* b,
                               const dg_store* sb, uint64_t* out_keys, uint64_t cap, u64* d_total) {
  const u64 g = e->diff_bsum_cap;
  u64* use = e->diff_bsum + (e->diff_parity ? g : 0);
  u64* zero = e->diff_bsum + (e->diff_parity ? 0 : g);
  e->diff_parity ^= 1;
  return launch_merkle_diff(merkle_of(a), rows_of(sa), merkle_of(b), rows_of(sb), out_keys, cap,
                            (u64*)e->tmp, use, zero, g, d_total, e->stream);
}

// pinned host staging (kernel descriptors, digit histograms), grown on demand
int ensure_stage(dg_engine* e, size_t bytes) {
  if (bytes <= e->h_stage_cap) return DG_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->h_stage) HIP_TRY(hipHostFree(e->h_stage));
  e->h_stage = nullptr;
  e->h_stage_cap = 0;
  if (hipHostMalloc(&e->h_stage, bytes, 0) != hipSuccess)
    return fail(DG_E_NOMEM, "pinned staging of %zu bytes failed", bytes);
  e->h_stage_cap = bytes;
  return DG_OK;
}

int ensure_counts(dg_engine* e, u64 tiles) {
  if (tiles <= e->counts_cap) return DG_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->counts) HIP_TRY(hipFree(e->counts));
  e->counts = nullptr;
  u64 cap = std::max<u64>(tiles, 4096);
  if (hipMalloc(&e->counts, cap * sizeof(u32)) != hipSuccess)
    return fail(DG_E_NOMEM, "hipMalloc of %llu tile-count granules failed", cap);
  HIP_TRY(hipMemsetAsync(e->counts, 0, cap * sizeof(u32), e->stream));  // epoch 0: never current
  e->counts_cap = cap;
  return DG_OK;
}

// A fresh epoch per look-back launch; granules of older epochs read as "not ready".
int next_scan(dg_engine* e, Scan* s) {
  if (++e->epoch >= (1u << 20)) {
    HIP_TRY(hipMemsetAsync(e->state, 0, e->state_cap * sizeof(u64), e->stream));
    if (e->counts) HIP_TRY(hipMemsetAsync(e->counts, 0, e->counts_cap * sizeof(u32), e->stream));
    HIP_TRY(hipMemsetAsync(e->started, 0, JOIN_MAX_GRID * sizeof(u32), e->stream));
    e->epoch = 1;
  }
  s->counts = e->counts;
  s->state = e->state;
  s->ticket = e->ticket;
  s->err = e->ticket + 1;
  s->started = e->started;
  s->abort = e->ticket + 4;
  s->epoch = e->epoch;
  return DG_OK;
}

// Copies the engine's counts and error words into mapped host memory, then publishes the
// call's sequence number (system scope, after a system fence): when the host sees the
// number, everything before this kernel on the stream has finished and the copies landed.
__global__ void publish_counts_kernel(const u64* d, u64* h, u64 seq) {
  const int l = threadIdx.x;
  if (l < 16) h[l] = d[l];  // d_counts[0..8) and ticket[0..16)
  __threadfence_system();
  __syncthreads();
  if (l == 0) __hip_atomic_store(h + 16, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The first n counts and the error bits (ticket[1]) of a synchronous call: d_counts[0..8)
// and ticket[0..2) are contiguous on the device and land in h_counts[0..9).  Instead of a
// D2H copy and a stream synchronize (≈ 14 µs on top of a config-2 join), a one-wave kernel
// publishes them into mapped host memory and the host polls its sequence word; past 20 ms
// (a long call) the runtime's synchronize takes over, and it is what reports a fault.
// wait_published: the host side alone, for a launch that publishes `seq` itself (the
// small join's tail kernel).
int wait_published(dg_engine* e, u64 seq) {
  const volatile u64* flag = e->h_pub + 16;
  const auto t0 = std::chrono::steady_clock::now();
  bool seen = false;
  for (u32 i = 0;; i++) {
    if (*flag == seq) {
      seen = true;
      break;
    }
    if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    __builtin_ia32_pause();
  }
  if (!seen) {
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (*flag != seq) return fail(DG_E_DEVICE, "counts were not published");
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  memcpy(e->h_counts, (const void*)e->h_pub, 8 * sizeof(u64) + 2 * sizeof(u32));
  memcpy(e->h_ticket, (const void*)(e->h_pub + 8), sizeof(e->h_ticket));
  return DG_OK;
}

int sync_words(dg_engine* e) {
  const u64 seq = ++e->pub_seq;
  hipLaunchKernelGGL(publish_counts_kernel, dim3(1), dim3(WAVE), 0, e->stream, e->d_counts, e->d_pub, seq);
  HIP_TRY(hipGetLastError());
  return wait_published(e, seq);
}

// ticket word: the Merkle kernels' arrival counter.  It is reset by the last workgroup of
// every build / update launch, not per launch.  A launch either runs every workgroup to
// that reset (the kernels never wait on another workgroup before arriving) or does not
// start at all (a launch error); a kernel that faults leaves the device unusable anyway.
// read_counts also zeroes it whenever a call reports error bits.
constexpr int MERKLE_ARRIVE = 6;
constexpr int CONT_HOME = 18;  // h_pub words [18, 24): dg_merkle_continue_home's result header
constexpr int TAIL_ARRIVE = 7;  // dg_join_delta_home's tail kernel: every workgroup arrives
constexpr int KD_ARRIVE = 8;    // dg_join_delta's count kernel: the last workgroup scans
constexpr int MUT_ARRIVE = 9;   // dg_mutate_batch's count kernel: the last tile scans
constexpr int SPL_ARRIVE = 10;  // dg_join_delta's moved-rows copy: the last workgroup publishes
constexpr int KD_ERR = 11;      // dg_join_delta's tree input-error word (zero between calls)

int published_errors(dg_engine* e);

int read_counts(dg_engine* e, int n) {
  (void)n;
  const int rc = sync_words(e);
  if (rc != DG_OK) return rc;
  return published_errors(e);
}

// the error bits of the count block just published (a look-back timeout, an aborted grid)
int published_errors(dg_engine* e) {
  e->last_err_bits = 0;
  u32 err = 0;
  memcpy(&err, (const char*)&e->h_counts[8] + sizeof(u32), sizeof(u32));
  if (err) {
    e->last_err_bits = err;
    HIP_TRY(hipMemsetAsync(e->ticket, 0, 4 * sizeof(u32), e->stream));
    HIP_TRY(hipMemsetAsync(e->ticket + MERKLE_ARRIVE, 0, 2 * sizeof(u32), e->stream));  // and TAIL_ARRIVE
    HIP_TRY(hipStreamSynchronize(e->stream));
    return fail(DG_E_DEVICE, "a kernel timed out or a join grid aborted (error bits 0x%x)", err);
  }
  return DG_OK;
}

Rows rows_of(const dg_store* s) {
  Rows r;
  r.key = s->key;
  r.val = s->val;
  r.ts = s->ts;
  r.node = s->node;
  r.cnt = s->cnt;
  r.n = s->n;
  return r;
}

RowsOut rows_out_of(dg_store* s) {
  RowsOut r;
  r.key = s->key;
  r.val = s->val;
  r.ts = s->ts;
  r.node = s->node;
  r.cnt = s->cnt;
  return r;
}

Ctx ctx_of(const dg_context* c) {
  Ctx x;
  x.node = c->node;
  x.cnt = c->cnt;
  x.n = c->n;
  x.kind = c->kind;
  return x;
}

int check_store(const dg_store* s, const char* what) {
  if (!s) return fail(DG_E_INVAL, "%s: null store", what);
  if (s->n && (!s->key || !s->val || !s->ts || !s->node || !s->cnt))
    return fail(DG_E_INVAL, "%s: null column with n=%llu", what, (unsigned long long)s->n);
  return DG_OK;
}

int check_ctx(const dg_context* c, const char* what) {
  if (!c) return fail(DG_E_INVAL, "%s: null context", what);
  if (c->kind != DG_CTX_VV && c->kind != DG_CTX_DOTS)
    return fail(DG_E_INVAL, "%s: bad context kind %d", what, c->kind);
  if (c->n && (!c->node || !c->cnt)) return fail(DG_E_INVAL, "%s: null context column", what);
  return DG_OK;
}

#define TRY(x)              \
  do {                      \
    int _r = (x);           \
    if (_r != DG_OK) return _r; \
  } while (0)

// Asynchronous calls logged for a replay at dg_engine_sync (a single-pass join grid that
// aborted for lack of residency).  A full log is settled before the next call is added.
constexpr size_t MAX_PENDING = 4096;

// Every synchronous entry point settles the asynchronous calls before it enqueues its own
// work: an aborted grid's error bit is then seen (and its calls replayed) by
// dg_engine_sync, never by the synchronous call's own error check, which would clear
// it and leave the aborted join's output unreported.
int settle(dg_engine* e) {
  if (!e->pending.empty()) return dg_engine_sync(e);
  return DG_OK;
}

int merkle_build_enqueue(dg_engine* e, const dg_store* s, dg_merkle* t, uint64_t* d_n_keys);

// chg (optional): the join also records its change events (dg_join2_changes); *chg
// receives their scratch for launch_join2_changes.
int join2_enqueue(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
                  const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
                  dg_context* out_ctx, uint64_t* d_counts, void** chg = nullptr,
                  bool force_two_pass = false) {
  TRY(check_store(a, "dg_join2 a"));
  TRY(check_store(b, "dg_join2 b"));
  TRY(check_ctx(ca, "dg_join2 ca"));
  TRY(check_ctx(cb, "dg_join2 cb"));
  if (!out || !out_ctx || !d_counts) return fail(DG_E_INVAL, "dg_join2: null output");
  if (keys == nullptr && n_keys != 0) return fail(DG_E_INVAL, "dg_join2: keys NULL with n_keys>0");
  if (out->cap < a->n + b->n)
    return fail(DG_E_CAPACITY, "dg_join2: out cap %llu < %llu rows in", (unsigned long long)out->cap,
                (unsigned long long)(a->n + b->n));
  if (out_ctx->cap < ca->n + cb->n)
    return fail(DG_E_CAPACITY, "dg_join2: out_ctx cap %llu < %llu", (unsigned long long)out_ctx->cap,
                (unsigned long long)(ca->n + cb->n));
  if (a->n + b->n && (!out->key || !out->val || !out->ts || !out->node || !out->cnt))
    return fail(DG_E_INVAL, "dg_join2: null output column");
  TRY(set_device(e));
  TRY(ensure_state(e, 3 * join2_tiles_cap(a->n, b->n) + 3));  // granules + tile + keyset splits
  const bool two_pass = (force_two_pass || e->join_mode == JOIN_TWO_PASS) && !chg;  // changes: single pass
  if (!two_pass) TRY(ensure_counts(e, join2_tiles_cap(a->n, b->n)));
  const size_t ctx_bytes = (ctx_union_tmp_bytes(ca->n, cb->n) + 255) / 256 * 256;
  const size_t pass_bytes = two_pass ? (join2_pass_tmp_bytes(a->n, b->n) + 255) / 256 * 256 : 0;
  const size_t chg_bytes = chg ? join2_changes_tmp_bytes(a->n, b->n) : 0;
  TRY(ensure_tmp(e, ctx_bytes + pass_bytes + chg_bytes));
  void* chg_tmp = chg ? (char*)e->tmp + ctx_bytes + pass_bytes : nullptr;
  if (chg) *chg = chg_tmp;
  Scan sc;
  TRY(next_scan(e, &sc));
  hipStream_t st = e->stream;
  hipStream_t ps = two_pass ? nullptr : shared_join_stream(e);
  if (ps) {
    HIP_TRY(hipEventRecord(e->ev_in, e->stream));
    HIP_TRY(hipStreamWaitEvent(ps, e->ev_in, 0));
    st = ps;
  }
  HIP_TRY(launch_join2(rows_of(a), ctx_of(ca), rows_of(b), ctx_of(cb), keys, keys ? n_keys : 0,
                       rows_out_of(out), out_ctx->node, out_ctx->cnt, e->tmp,
                       (char*)e->tmp + ctx_bytes, two_pass ? JOIN_TWO_PASS : JOIN_SINGLE_PASS,
                       sc, e->join_workers, d_counts, st, chg_tmp));
  if (ps) {
    HIP_TRY(hipEventRecord(e->ev_out, ps));
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_out, 0));
  }
  out_ctx->kind = (ca->kind == DG_CTX_DOTS && cb->kind == DG_CTX_DOTS) ? DG_CTX_DOTS : DG_CTX_VV;
  return DG_OK;
}

MerkleT merkle_of(const dg_merkle* t);
int check_merkle(const dg_merkle* t, const char* what);
int input_error(dg_engine* e, const char* what);

// Engine scratch that persists across calls (the fold's ping-pong states; the splice's
// taken rows, edit and index), grown on demand.
int ensure_buf(dg_engine* e, void** buf, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return DG_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (*buf) HIP_TRY(hipFree(*buf));
  *buf = nullptr;
  *cap = 0;
  if (hipMalloc(buf, bytes) != hipSuccess)
    return fail(DG_E_NOMEM, "hipMalloc of %zu scratch bytes failed", bytes);
  *cap = bytes;
  return DG_OK;
}

// A store of `rows` rows carved from p (columns 256-B aligned); advances p.
dg_store carve_store(char*& p, u64 rows) {
  auto take = [&](size_t bytes) {
    char* q = p;
    p += (bytes + 255) / 256 * 256;
    return q;
  };
  dg_store s{};
  s.key = (uint64_t*)take(rows * 8);
  s.val = (uint64_t*)take(rows * 8);
  s.ts = (int64_t*)take(rows * 8);
  s.cnt = (uint64_t*)take(rows * 8);
  s.node = (uint32_t*)take(rows * 4);
  s.cap = rows;
  s.n = 0;
  return s;
}

// A keyed join whose delta and keyset are small against the state (CausalCrdt's sync
// deltas, causal_crdt.ex:383-384) as a splice (csrc/splice.hip): the state's rows of the
// keyset are taken out, joined with the delta on the join kernels, and the output is
// written in one streaming pass (the untouched rows moved, the joined keys' rows in the
// holes).  *done = false (and nothing of the caller's changed) when the splice does not
// apply: the delta holds a key outside the keyset (its right-biased carry would replace
// state rows the splice keeps), the taken rows exceed their bound, or the join grid
// aborted; the caller then runs the full join.  Synchronous (two host syncs).
// (the splice moves rows in 16-byte pairs: the state's and the output's 8-byte columns
// must be 16-byte aligned, their node columns 8-byte aligned)
bool pair_aligned(const void* k, const void* v, const void* t, const void* n, const void* c) {
  return !(((uintptr_t)k | (uintptr_t)v | (uintptr_t)t | (uintptr_t)c) & 15) && !((uintptr_t)n & 7);
}

bool splice_wanted(const dg_engine* e, const dg_store* a, const dg_store* b, const uint64_t* keys,
                   uint64_t n_keys, const dg_store* out) {
  return e->splice && keys && n_keys > 0 && (n_keys + b->n) * 8 <= a->n && out &&
         pair_aligned(a->key, a->val, a->ts, a->node, a->cnt) &&
         pair_aligned(out->key, out->val, out->ts, out->node, out->cnt);
}

// The splice's scratch (e->spl): the state's rows of the keyset (ak), the edit (ed),
// the per-key index and the per-tile entry ranges; and a context for the join's union.
struct Splice {
  dg_store ak, ed;
  dg_context uctx;
  SpliceArgs sp;
  u64 n_ak = 0;
};

// Phase 1: take the state's rows of the keyset (with the per-key index) and check that
// every key of the delta is in the keyset.  *ok = false: the splice does not apply (the
// full join does).  One host sync.
int splice_take(dg_engine* e, const dg_store* a, const dg_store* b, const uint64_t* keys,
                uint64_t n_keys, u64 uctx_cap, Splice* w, bool* ok) {
  *ok = false;
  const u64 cap_k = std::min<u64>(a->n, 16 * n_keys + 4096);  // taken rows: a few per key
  const u64 cap_e = cap_k + b->n;
  const size_t idx_bytes = ((n_keys + 1) * 8 + 255) / 256 * 256;
  const size_t tile_bytes = ((splice_tiles(a->n) + 1) * 8 + 255) / 256 * 256;
  const size_t ctx_bytes = (uctx_cap * 12 + 2 * 256) / 256 * 256 + 256;
  const size_t bytes = ((cap_k * 36 + 5 * 256) + (cap_e * 36 + 5 * 256) + 5 * idx_bytes +
                        tile_bytes + ctx_bytes + 256 + 255) / 256 * 256;
  TRY(ensure_buf(e, &e->spl, &e->spl_cap, bytes));
  char* p = (char*)e->spl;
  w->ak = carve_store(p, cap_k);
  w->ed = carve_store(p, cap_e);
  SpliceArgs& sp = w->sp;
  sp = SpliceArgs{};
  sp.a_lo = (u64*)p;
  sp.a_off = (u64*)(p + idx_bytes);
  sp.end = (u64*)(p + 2 * idx_bytes);
  sp.shift = (i64*)(p + 3 * idx_bytes);
  sp.gap = (i64*)(p + 4 * idx_bytes);
  p += 5 * idx_bytes;
  sp.tile_u0 = (u64*)p;
  p += tile_bytes;
  w->uctx = dg_context{};
  w->uctx.cnt = (uint64_t*)p;
  w->uctx.node = (uint32_t*)(p + (uctx_cap * 8 + 255) / 256 * 256);
  w->uctx.cap = uctx_cap;
  p += ctx_bytes;
  sp.moved = (u32*)(e->d_counts + 5);  // zeroed with n_ak and bad below
  TRY(ensure_state(e, take_tiles(n_keys) + 2));
  Scan sc;
  TRY(next_scan(e, &sc));
  HIP_TRY(hipMemsetAsync(e->d_counts + 3, 0, 3 * sizeof(u64), e->stream));  // n_ak, bad, moved
  // the keyset's rows: one search per key, or -- once the keys are dense enough that the
  // searches' scattered lines outweigh reading every key -- one streaming pass over the
  // state's keys (the located ranges go through `end`, which the index overwrites later).
  // At 1 key in 100 rows (config 4) both take 60 us for 12.5M rows; the searches grow
  // with the keys, the pass does not.
  u32* pre_len = nullptr;
  if (n_keys * 60 >= a->n) {
    pre_len = (u32*)sp.end;
    HIP_TRY(launch_splice_locate(rows_of(a), keys, n_keys, (u64*)sp.a_lo, pre_len, e->stream));
  }
  HIP_TRY(launch_take_keys(rows_of(a), keys, n_keys, rows_out_of(&w->ak), cap_k, sc,
                           e->d_counts + 3, e->stream, (u64*)sp.a_lo, (u64*)sp.a_off, pre_len));
  HIP_TRY(launch_splice_check(b->key, b->n, keys, n_keys, e->d_counts + 4, e->stream));
  TRY(read_counts(e, 5));
  w->n_ak = e->h_counts[3];
  if (e->h_counts[4] != 0 || w->n_ak > cap_k) return DG_OK;
  w->ak.n = w->n_ak;
  sp.a = rows_of(a);
  sp.keys = keys;
  sp.nk = n_keys;
  sp.e = rows_of(&w->ed);
  sp.e.n = w->n_ak + b->n;  // a bound: the kernels read the count
  sp.d_ne = e->d_counts;
  *ok = true;
  return DG_OK;
}

// Phase 2: the edit E = join(taken rows, delta, keys) (+ its changed keys) and the index.
int splice_edit(dg_engine* e, Splice* w, const dg_context* ca, const dg_store* b,
                const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_context* out_ctx,
                bool with_changes, uint64_t* changed, uint64_t cap) {
  void* chg = nullptr;
  TRY(join2_enqueue(e, &w->ak, ca, b, cb, keys, n_keys, &w->ed, out_ctx, e->d_counts,
                    with_changes ? &chg : nullptr));
  if (with_changes)
    HIP_TRY(launch_join2_changes(w->ak.n, b->n, chg, changed, cap, e->d_counts + 2, e->stream));
  HIP_TRY(launch_splice_index(w->sp, e->stream));
  return DG_OK;
}

int splice_join(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
                const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
                dg_context* out_ctx, bool with_changes, uint64_t* changed, uint64_t cap,
                uint64_t* n_changed, bool* done) {
  *done = false;
  TRY(check_store(a, "dg_join2 a"));
  TRY(check_store(b, "dg_join2 b"));
  TRY(check_ctx(ca, "dg_join2 ca"));
  TRY(check_ctx(cb, "dg_join2 cb"));
  if (!out || !out_ctx) return fail(DG_E_INVAL, "dg_join2: null output");
  if (out->cap < a->n + b->n)
    return fail(DG_E_CAPACITY, "dg_join2: out cap %llu < %llu rows in", (unsigned long long)out->cap,
                (unsigned long long)(a->n + b->n));
  if (!out->key || !out->val || !out->ts || !out->node || !out->cnt)
    return fail(DG_E_INVAL, "dg_join2: null output column");
  TRY(set_device(e));
  Splice w;
  bool ok = false;
  TRY(splice_take(e, a, b, keys, n_keys, 0, &w, &ok));
  if (!ok) return DG_OK;  // the full join applies
  TRY(splice_edit(e, &w, ca, b, cb, keys, n_keys, out_ctx, with_changes, changed, cap));
  w.sp.out = rows_out_of(out);
  HIP_TRY(launch_splice_copy(w.sp, false, e->stream));
  if (read_counts(e, 3) != DG_OK) return DG_OK;  // a grid aborted: the full join re-runs
  out->n = a->n - w.n_ak + e->h_counts[0];
  out_ctx->n = e->h_counts[1];
  if (n_changed) *n_changed = e->h_counts[2];
  *done = true;
  return DG_OK;
}

// MerkleMap put/delete + update_hashes of `keys` (the tree indexes `olds`; afterwards
// `news`), all or nothing: when the update meets an input error (a changed key outside the
// tree's shard, a bucket over 65535 rows) the same update with the stores exchanged
// restores every node and count bit for bit, and the error is returned.  `ready`: the
// dirty flags, key-count shards and error word are zeroed already (dg_join_delta's
// set-up launch).  `tail` (optional) enqueues work between the update and its host sync
// that must not take effect after a failed update (it reads the error word as a guard).
// *d_n_keys = the change in distinct keys (not applied to t->n_keys).
template <class Tail>
int tree_update(dg_engine* e, dg_merkle* t, const dg_store* olds, const dg_store* news,
                const uint64_t* keys, uint64_t n_keys, const char* what, bool ready, Tail tail,
                u64* d_n_keys) {
  // scratch: the hand-off words | dirty flags (u32, padded to even) | the per-chunk
  // row-count changes (i64, for the chunk starts); dirty and cdelta zeroed in one launch
  const u64 chunks = merkle_chunks(t->depth), cw = merkle_ctr_words(t->depth);
  const u64 cpad = (chunks + 1) & ~1ull, zw = cpad + 2 * chunks;
  TRY(ensure_tmp(e, (cw + zw) * sizeof(u32)));
  u64* hand = (u64*)e->tmp;
  u32* dirty = (u32*)e->tmp + cw;
  i64* cdelta = (i64*)(dirty + cpad);
  if (!ready)
    HIP_TRY(launch_splice_finish(nullptr, nullptr, 0, nullptr, nullptr, dirty, zw, e->d_counts,
                                 e->ticket + 3, e->stream));
  HIP_TRY(launch_merkle_update(merkle_of(t), rows_of(olds), rows_of(news), keys, n_keys, dirty,
                               e->d_counts, e->ticket + MERKLE_ARRIVE, hand, cdelta, e->ticket + 3,
                               e->stream));
  TRY(tail());
  TRY(read_counts(e, 8));
  u64 dk = 0;
  for (int i = 0; i < 8; i++) dk += e->h_counts[i];  // signed changes, two's complement
  *d_n_keys = dk;
  if (!(e->h_ticket[3] & MERKLE_INPUT_ERR)) return DG_OK;
  const int rc = input_error(e, what);
  const std::string msg = g_err;
  HIP_TRY(launch_splice_finish(nullptr, nullptr, 0, nullptr, nullptr, dirty, zw, e->d_counts,
                               e->ticket + 3, e->stream));
  HIP_TRY(launch_merkle_update(merkle_of(t), rows_of(news), rows_of(olds), keys, n_keys, dirty,
                               e->d_counts, e->ticket + MERKLE_ARRIVE, hand, cdelta, e->ticket + 3,
                               e->stream));
  HIP_TRY(hipMemsetAsync(e->ticket + 3, 0, sizeof(u32), e->stream));  // the undo's own bits
  TRY(read_counts(e, 0));
  g_err = msg;
  return rc;
}

int tree_update(dg_engine* e, dg_merkle* t, const dg_store* olds, const dg_store* news,
                const uint64_t* keys, uint64_t n_keys, const char* what) {
  u64 dk = 0;
  TRY(tree_update(e, t, olds, news, keys, n_keys, what, false, [] { return (int)DG_OK; }, &dk));
  t->n_keys += dk;
  return DG_OK;
}

}  // namespace

extern "C" {

int dg_abi_version(void) { return DG_ABI_VERSION; }

const char* dg_last_error(void) { return g_err.c_str(); }

int dg_engine_create(int device, void* hip_stream, dg_engine** out) {
  if (!out) return fail(DG_E_INVAL, "dg_engine_create: null out");
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return fail(DG_E_INVAL, "dg_engine_create: device %d of %d", device, ndev);
  dg_engine* e = new dg_engine();
  e->device = device;
  {
    const char* v = getenv("DG_JOIN_WORKERS");
    if (v && atoi(v) > 0) e->join_workers = atoi(v);
    const char* m = getenv("DG_JOIN_MODE");
    if (m && m[0] == '2') e->join_mode = JOIN_TWO_PASS;
    const char* sp = getenv("DG_SPLICE");
    if (sp && sp[0] == '0') e->splice = false;
    const char* kd = getenv("DG_KD");
    if (kd && kd[0] == '0') e->kd = false;
    const char* am = getenv("DG_APPLY_MODE");
    if (am && strcmp(am, "fold") == 0) e->apply_mode = 1;
    if (am && strcmp(am, "onepass") == 0) e->apply_mode = 2;
  }
  int rc = set_device(e);
  if (rc != DG_OK) {
    delete e;
    return rc;
  }
  if (hip_stream) {
    e->stream = (hipStream_t)hip_stream;
  } else {
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
      delete e;
      return fail(DG_E_DEVICE, "hipStreamCreate failed");
    }
    e->own_stream = true;
  }
  if (hipMalloc(&e->d_counts, 8 * sizeof(u64) + 16 * sizeof(u32)) != hipSuccess ||
      hipMalloc(&e->started, JOIN_MAX_GRID * sizeof(u32)) != hipSuccess ||
      hipHostMalloc(&e->h_counts, 16 * sizeof(u64), 0) != hipSuccess ||
      hipHostMalloc(&e->h_pub, 24 * sizeof(u64), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&e->d_pub, e->h_pub, 0) != hipSuccess) {
    dg_engine_destroy(e);
    return fail(DG_E_NOMEM, "dg_engine_create: allocation failed");
  }
  e->ticket = (u32*)(e->d_counts + 8);
  memset(e->h_pub, 0, 24 * sizeof(u64));  // sequence 0: nothing published yet
  if (hipMemsetAsync(e->d_counts, 0, 8 * sizeof(u64) + 16 * sizeof(u32), e->stream) != hipSuccess ||
      hipMemsetAsync(e->started, 0, JOIN_MAX_GRID * sizeof(u32), e->stream) != hipSuccess) {
    dg_engine_destroy(e);
    return fail(DG_E_DEVICE, "dg_engine_create: hipMemsetAsync failed");
  }
  rc = ensure_state(e, 4096);
  if (rc != DG_OK) {
    dg_engine_destroy(e);
    return rc;
  }
  if (hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_out, hipEventDisableTiming) != hipSuccess) {
    dg_engine_destroy(e);
    return fail(DG_E_DEVICE, "dg_engine_create: hipEventCreate failed");
  }
  {
    std::lock_guard<std::mutex> g(g_share_mu);
    const int n = ++g_share[device & 63].engines;
    // the first engine's joins ran on its own stream: let them finish before any join of
    // this one can start, from here on they share a stream
    if (n == 2) hipDeviceSynchronize();
  }
  *out = e;
  return DG_OK;
}

int dg_engine_destroy(dg_engine* e) {
  if (!e) return DG_OK;
  hipSetDevice(e->device);
  if (e->stream) hipStreamSynchronize(e->stream);
  if (e->state) hipFree(e->state);
  if (e->d_counts) hipFree(e->d_counts);
  if (e->h_counts) hipHostFree(e->h_counts);
  if (e->h_pub) hipHostFree(e->h_pub);
  if (e->tmp) hipFree(e->tmp);
  if (e->counts) hipFree(e->counts);
  if (e->started) hipFree(e->started);
  if (e->fold) hipFree(e->fold);
  if (e->spl) hipFree(e->spl);
  if (e->ubuf) hipFree(e->ubuf);
  if (e->sml) hipFree(e->sml);
  if (e->kdb) hipFree(e->kdb);
  if (e->kdz) hipFree(e->kdz);
  if (e->diff_bsum) hipFree(e->diff_bsum);
  if (e->h_stage) hipHostFree(e->h_stage);
  if (e->own_stream && e->stream) hipStreamDestroy(e->stream);
  if (e->ev_in || e->ev_out) {  // a registered engine (creation got past the registry)
    if (e->ev_in) hipEventDestroy(e->ev_in);
    if (e->ev_out) hipEventDestroy(e->ev_out);
    std::lock_guard<std::mutex> g(g_share_mu);
    DevShare& d = g_share[e->device & 63];
    if (e->ev_out && --d.engines == 0 && d.stream) {
      hipStreamSynchronize(d.stream);
      hipStreamDestroy(d.stream);
      d.stream = nullptr;
    }
  }
  delete e;
  return DG_OK;
}

void* dg_engine_stream(dg_engine* e) { return e ? (void*)e->stream : nullptr; }

constexpr int RETRY_WORKERS = 32;  // dg_join2_changes' re-run after an aborted grid

// Error bits of the work on the engine stream so far (synchronizes), cleared.
static int stream_error(dg_engine* e, u32* err) {
  TRY(sync_words(e));
  *err = e->h_ticket[1];
  if (*err) {
    HIP_TRY(hipMemsetAsync(e->ticket, 0, 4 * sizeof(u32), e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  return DG_OK;
}

int dg_engine_sync(dg_engine* e) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(set_device(e));
  u32 err = 0;
  TRY(stream_error(e, &err));
  if (err & 3u) {
    // a single-pass join grid aborted (not co-resident) or timed out: replay the
    // asynchronous calls since the last sync in order, the joins on the two-pass kernels
    // (their workgroups never wait on each other)
    std::vector<dg_engine::Pending> log;
    log.swap(e->pending);
    for (dg_engine::Pending& q : log) {
      if (q.kind == 0)
        TRY(join2_enqueue(e, &q.a, &q.ca, &q.b, &q.cb, q.keys, q.n_keys, &q.out, &q.out_ctx,
                          q.d_counts, nullptr, true));
      else
        TRY(merkle_build_enqueue(e, &q.a, q.tp, q.d_counts));
    }
    e->pending.clear();
    TRY(stream_error(e, &err));
  }
  e->pending.clear();
  if (err) return fail(DG_E_DEVICE, "kernel error bits 0x%x after dg_engine_sync", err);
  return DG_OK;
}

int dg_store_check(dg_engine* e, const dg_store* s) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_store(s, "dg_store_check"));
  TRY(set_device(e));
  TRY(settle(e));
  HIP_TRY(hipMemsetAsync(e->ticket + 2, 0, sizeof(u32), e->stream));
  HIP_TRY(launch_store_check(rows_of(s), e->ticket + 2, e->stream));
  TRY(sync_words(e));
  if (e->h_ticket[2]) return fail(DG_E_ORDER, "store rows are not strictly ascending");
  return DG_OK;
}

int dg_join2_async(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
                   const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
                   dg_context* out_ctx, uint64_t* d_counts) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (e->pending.size() >= MAX_PENDING) TRY(dg_engine_sync(e));
  TRY(join2_enqueue(e, a, ca, b, cb, keys, n_keys, out, out_ctx, d_counts));
  dg_engine::Pending q{};
  q.kind = 0;
  q.a = *a;
  q.b = *b;
  q.out = *out;
  q.ca = *ca;
  q.cb = *cb;
  q.out_ctx = *out_ctx;
  q.keys = keys;
  q.n_keys = n_keys;
  q.d_counts = d_counts;
  e->pending.push_back(q);
  return DG_OK;
}

int dg_join2(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
             const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
             dg_context* out_ctx) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(settle(e));  // earlier asynchronous calls
  if (splice_wanted(e, a, b, keys, n_keys, out)) {
    bool done = false;
    TRY(splice_join(e, a, ca, b, cb, keys, n_keys, out, out_ctx, false, nullptr, 0, nullptr, &done));
    if (done) return DG_OK;
  }
  TRY(join2_enqueue(e, a, ca, b, cb, keys, n_keys, out, out_ctx, e->d_counts));
  if (read_counts(e, 2) != DG_OK) {
    // a single-pass grid that could not become resident (another process's persistent
    // kernels on this GPU) timed out: the two-pass kernels never wait on each other
    TRY(join2_enqueue(e, a, ca, b, cb, keys, n_keys, out, out_ctx, e->d_counts, nullptr, true));
    TRY(read_counts(e, 2));
  }
  out->n = e->h_counts[0];
  out_ctx->n = e->h_counts[1];
  return DG_OK;
}

int dg_join2_changes(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
                     const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
                     dg_context* out_ctx, uint64_t* changed, uint64_t cap, uint64_t* n_changed) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (!n_changed || (cap && !changed)) return fail(DG_E_INVAL, "dg_join2_changes: null output");
  TRY(settle(e));
  if (splice_wanted(e, a, b, keys, n_keys, out)) {
    bool done = false;
    TRY(splice_join(e, a, ca, b, cb, keys, n_keys, out, out_ctx, true, changed, cap, n_changed, &done));
    if (done) {
      if (*n_changed > cap)
        return fail(DG_E_CAPACITY, "dg_join2_changes: %llu changed keys > cap %llu",
                    (unsigned long long)*n_changed, (unsigned long long)cap);
      return DG_OK;
    }
  }
  void* chg = nullptr;
  TRY(join2_enqueue(e, a, ca, b, cb, keys, n_keys, out, out_ctx, e->d_counts, &chg));
  HIP_TRY(launch_join2_changes(a->n, b->n, chg, changed, cap, e->d_counts + 2, e->stream));
  if (read_counts(e, 3) != DG_OK) {
    // the grid aborted (not co-resident): the change events come from the single-pass
    // kernel only, so re-run it on a grid small enough to find room beside other work
    const int workers = e->join_workers;
    e->join_workers = RETRY_WORKERS;
    const int rc = join2_enqueue(e, a, ca, b, cb, keys, n_keys, out, out_ctx, e->d_counts, &chg);
    e->join_workers = workers;
    TRY(rc);
    HIP_TRY(launch_join2_changes(a->n, b->n, chg, changed, cap, e->d_counts + 2, e->stream));
    TRY(read_counts(e, 3));
  }
  out->n = e->h_counts[0];
  out_ctx->n = e->h_counts[1];
  *n_changed = e->h_counts[2];
  if (*n_changed > cap)
    return fail(DG_E_CAPACITY, "dg_join2_changes: %llu changed keys > cap %llu",
                (unsigned long long)*n_changed, (unsigned long long)cap);
  return DG_OK;
}

// dg_join_delta_rows' output: the changed keys' rows of `src`; more than rows->cap is
// reported in rows->n, not as an error (the join before it is complete).  It runs after
// the join is committed, so any failure of the gather is reported the same way -- "rows
// not written" (rows->n > rows->cap) -- and never as an error of a join that applied.
static int take_changed_rows(dg_engine* e, const dg_store* src, const uint64_t* changed,
                             uint64_t n_changed, dg_store* rows) {
  const int rc = dg_take_keys(e, src, changed, n_changed, rows);
  if (rc == DG_E_CAPACITY) return DG_OK;
  if (rc != DG_OK) rows->n = rows->cap + 1;
  return DG_OK;
}

// dg_join_delta's one-wait path (kdelta.hip): count + scan, the context union, the tree's
// put/delete and re-reduction, the write (in place, or into `spare` with the moved rows'
// copy behind it), then ONE publish and wait.  *done = false and nothing changed when the
// delta has a row outside the keyset (the full join applies) or a key has more than KD_RUN
// rows on a side (the splice applies); a tree input error is undone before it returns.
static int kd_join_delta(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                         const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys, dg_store* spare,
                         dg_merkle* tree, uint64_t* changed, uint64_t cap, uint64_t* n_changed, int* swapped,
                         dg_store* rows, dg_context* ctx_out, bool* done) {
  *done = false;
  if (!e->kd || n_keys == 0 || state_ctx->kind != DG_CTX_VV || state->cap < state->n ||
      !pair_aligned(state->key, state->val, state->ts, state->node, state->cnt) ||
      !pair_aligned(spare->key, spare->val, spare->ts, spare->node, spare->cnt))
    return DG_OK;
  const u64 nk = n_keys, ntiles = (nk + KD_BLOCK - 1) / KD_BLOCK, a_tiles = splice_tiles(state->n);
  const u64 uctx_cap = state_ctx->n + delta_ctx->n;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t per_key = al(nk * 8), per_key1 = al((nk + 1) * 8), tiles_b = al(ntiles * KD_NV * 8);
  const size_t uc_b = al(uctx_cap * 8) + al(uctx_cap * 4), cu_b = al(ctx_union_tmp_bytes(state_ctx->n, delta_ctx->n));
  const size_t bytes = 7 * per_key + per_key1 + tiles_b + al((a_tiles + 2) * 8) + uc_b + cu_b;
  TRY(ensure_buf(e, &e->kdb, &e->kdb_cap, bytes));
  char* q = (char*)e->kdb;
  auto take = [&](size_t b) {
    char* r = q;
    q += b;
    return r;
  };
  KdArgs p{};
  p.a = rows_of(state);
  p.aw = rows_out_of(state);
  p.ca = ctx_of(state_ctx);
  p.ca_node = state_ctx->node;
  p.ca_cnt = state_ctx->cnt;
  p.ca_cap = state_ctx->cap;
  p.d = rows_of(delta);
  p.cd = ctx_of(delta_ctx);
  p.keys = keys;
  p.nk = nk;
  p.a_lo = (u64*)take(per_key);
  p.d_lo = (u64*)take(per_key);
  p.runs = (u64*)take(per_key);
  p.amask = (u64*)take(per_key);
  p.dmask = (u64*)take(per_key);
  p.dh = (u64*)take(per_key);
  p.end = (u64*)take(per_key);
  p.shift = (i64*)take(per_key1);
  p.part = (u64*)take(tiles_b);
  p.tile_u0 = (u64*)take(al((a_tiles + 2) * 8));
  u64* uc_cnt = (u64*)take(al(uctx_cap * 8));
  u32* uc_node = (u32*)take(al(uctx_cap * 4));
  void* cu_tmp = take(cu_b);
  p.uc_node = uc_node;
  p.uc_cnt = uc_cnt;
  p.ntiles = ntiles;
  p.changed = changed;
  p.cap = cap;
  p.has_rows = rows != nullptr;
  if (rows) {
    p.rows = rows_out_of(rows);
    p.rows_cap = rows->cap;
  }
  p.sp = rows_out_of(spare);
  if (ctx_out) {
    p.co_node = ctx_out->node;
    p.co_cnt = ctx_out->cnt;
    p.co_cap = ctx_out->cap;
  }
  p.a_tiles = a_tiles;
  p.has_tree = tree != nullptr;
  if (tree) p.t = merkle_of(tree);
  p.d_counts = e->d_counts;
  p.arrive = e->ticket + KD_ARRIVE;
  // the tree update's scratch: hand-off words (engine scratch), and the dirty flags and
  // chunk row-count changes in a buffer of their own that stays zero between calls
  u32* dirty = nullptr;
  u64* hand = nullptr;
  i64* cdelta = nullptr;
  u64 zw = 0;
  u32* err = e->ticket + KD_ERR;
  p.err = err;
  if (tree) {
    const u64 chunks = merkle_chunks(tree->depth), cw = merkle_ctr_words(tree->depth);
    const u64 cpad = (chunks + 1) & ~1ull;
    zw = cpad + 2 * chunks;
    TRY(ensure_tmp(e, cw * sizeof(u32)));
    hand = (u64*)e->tmp;
    if (zw * sizeof(u32) > e->kdz_cap) {
      TRY(ensure_buf(e, &e->kdz, &e->kdz_cap, zw * sizeof(u32)));
      HIP_TRY(hipMemsetAsync(e->kdz, 0, e->kdz_cap, e->stream));
    }
    dirty = (u32*)e->kdz;
    cdelta = (i64*)(dirty + cpad);
  }
  p.dirty = dirty;
  p.cdelta = cdelta;
  p.cu_tmp = cu_tmp;
  // three launches, one wait: the count (the per-key joins, the tree's put/delete, the scan
  // and the context union by its last workgroup), the write beside the tree's re-reduction,
  // the moved rows' copy (its last workgroup publishes the count block)
  HIP_TRY(launch_kd_join(p, e->stream));
  HIP_TRY(launch_kd_finish(p, dirty, e->ticket + MERKLE_ARRIVE, hand, cdelta, e->stream));
  SpliceArgs sp{};
  sp.a = rows_of(state);
  sp.keys = keys;
  sp.nk = nk;
  sp.a_lo = p.a_lo;
  sp.end = p.end;
  sp.shift = p.shift;
  sp.tile_u0 = p.tile_u0;
  sp.out = rows_out_of(spare);
  sp.run_if = e->d_counts + 5;  // rows moved
  sp.kguard = e->d_counts + 4;
  sp.h_pub = e->d_pub;
  sp.pub_counts = e->d_counts;
  sp.seq = ++e->pub_seq;
  sp.arrive_all = e->ticket + SPL_ARRIVE;
  HIP_TRY(launch_splice_move(sp, e->stream));
  TRY(wait_published(e, sp.seq));
  TRY(published_errors(e));
  const u64 g = e->h_counts[4];
  const u32 tbits = e->h_ticket[KD_ERR];
  if (g || (tbits & MERKLE_INPUT_ERR)) {
    // nothing of the state or its context was written (the write kernel saw the guard or
    // the error word), but the count kernel put the changes into the tree: the same update
    // with the opposite sign restores every bucket node and count bit for bit
    const int rc = (g & (KD_BAD | KD_BIG)) ? DG_OK
                   : (g & KD_CAP) ? fail(DG_E_CAPACITY, "dg_join_delta: %llu changed keys > cap %llu",
                                         (unsigned long long)e->h_counts[2], (unsigned long long)cap)
                  : (tbits & MERKLE_ERR_SHARD) ? fail(DG_E_INVAL, "dg_join_delta: a key outside the tree's shard")
                                  : fail(DG_E_CAPACITY, "dg_join_delta: a bucket holds more than 65535 rows "
                                                        "(use a deeper tree)");
    const std::string msg = g_err;
    if (tree) {  // (dirty and cdelta are zero again: the re-reduction consumed them)
      HIP_TRY(launch_kd_tree(merkle_of(tree), keys, p.runs, p.dh, nk, nullptr, -1, dirty,
                             e->ticket + MERKLE_ARRIVE, hand, cdelta, err, e->stream));
      HIP_TRY(hipMemsetAsync(err, 0, sizeof(u32), e->stream));  // (the undo's own bits too)
      TRY(read_counts(e, 0));
    }
    g_err = msg;
    return rc;  // (DG_OK with *done false: a delta row outside the keyset or a long key run --
                // the full join or the splice applies)
  }
  const u64 n_e = e->h_counts[0], n_chg = e->h_counts[2], n_rows = e->h_counts[3];
  const u64 n_ak = e->h_counts[6], dk = e->h_counts[7];
  if (e->h_counts[5]) {  // rows moved: the state is in `spare`
    const u64 n = state->n - n_ak + n_e;
    std::swap(*state, *spare);
    state->n = n;
    *swapped = 1;
  }
  state_ctx->n = e->h_counts[1];
  state_ctx->kind = DG_CTX_VV;
  if (tree) tree->n_keys += dk;
  *n_changed = n_chg;
  if (rows) rows->n = n_rows;  // (more than rows->cap: not written, as the caller's contract says)
  if (ctx_out) {
    ctx_out->n = state_ctx->n;  // (more than ctx_out->cap: not written)
    ctx_out->kind = DG_CTX_VV;
  }
  *done = true;
  return DG_OK;
}

// dg_join_delta[_rows]: rows (optional) receives the changed keys' joined rows
// ctx_out (optional): a copy of the joined context
static int join_delta_core(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                           const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                           dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                           uint64_t* n_changed, int* swapped, dg_store* rows, dg_context* ctx_out, bool* kd_done) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (!swapped || !n_changed || (cap && !changed) || !spare || !state || !state_ctx)
    return fail(DG_E_INVAL, "dg_join_delta: null argument");
  *swapped = 0;
  *n_changed = 0;
  TRY(check_store(state, "dg_join_delta state"));
  TRY(check_store(delta, "dg_join_delta delta"));
  TRY(check_ctx(state_ctx, "dg_join_delta state_ctx"));
  TRY(check_ctx(delta_ctx, "dg_join_delta delta_ctx"));
  if (tree) TRY(check_merkle(tree, "dg_join_delta tree"));
  if (keys == nullptr && n_keys != 0) return fail(DG_E_INVAL, "dg_join_delta: keys NULL with n_keys>0");
  if (spare->cap < state->n + delta->n)
    return fail(DG_E_CAPACITY, "dg_join_delta: spare cap %llu < %llu rows in",
                (unsigned long long)spare->cap, (unsigned long long)(state->n + delta->n));
  if (state_ctx->cap < state_ctx->n + delta_ctx->n)
    return fail(DG_E_CAPACITY, "dg_join_delta: state_ctx cap %llu < %llu",
                (unsigned long long)state_ctx->cap, (unsigned long long)(state_ctx->n + delta_ctx->n));
  TRY(set_device(e));
  TRY(settle(e));
  // All or nothing: nothing of *state, *state_ctx or the tree changes unless the call
  // succeeds.  Everything that can fail (the join's grid, the capacity of `changed`, the
  // tree update's input checks) runs on scratch and `spare` first; the state is written
  // last, by kernels that skip their writes when the tree update reported an error.
  const u64 uctx_cap = state_ctx->n + delta_ctx->n;
  const dg_context_kind out_kind =
      (state_ctx->kind == DG_CTX_DOTS && delta_ctx->kind == DG_CTX_DOTS) ? DG_CTX_DOTS : DG_CTX_VV;
  {
    bool done = false;
    TRY(kd_join_delta(e, state, state_ctx, delta, delta_ctx, keys, n_keys, spare, tree, changed, cap,
                      n_changed, swapped, rows, ctx_out, &done));
    *kd_done = done;
    if (done) return DG_OK;
  }
  Splice w;
  bool ok = false;
  const dg_store old_state = *state;
  if (splice_wanted(e, state, delta, keys, n_keys, spare) && state->cap >= state->n)
    TRY(splice_take(e, state, delta, keys, n_keys, uctx_cap, &w, &ok));
  if (!ok) {
    // the full keyed join into the spare store (the merge, or a splice into `spare` that
    // dg_join2_changes picks itself), the context into its own scratch, then the tree
    TRY(ensure_buf(e, &e->ubuf, &e->ubuf_cap, (uctx_cap * 12 + 1024 + 255) / 256 * 256));
    dg_context uc{};
    uc.cnt = (uint64_t*)e->ubuf;
    uc.node = (uint32_t*)((char*)e->ubuf + (uctx_cap * 8 + 255) / 256 * 256);
    uc.cap = uctx_cap;
    TRY(dg_join2_changes(e, state, state_ctx, delta, delta_ctx, keys, n_keys, spare, &uc,
                         changed, cap, n_changed));
    if (tree) TRY(tree_update(e, tree, &old_state, spare, changed, *n_changed, "dg_join_delta"));
    HIP_TRY(hipMemcpyAsync(state_ctx->node, uc.node, uc.n * 4, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(state_ctx->cnt, uc.cnt, uc.n * 8, hipMemcpyDeviceToDevice, e->stream));
    TRY(read_counts(e, 0));
    state_ctx->n = uc.n;
    state_ctx->kind = uc.kind;
    std::swap(*state, *spare);
    *swapped = 1;
    if (rows) TRY(take_changed_rows(e, state, changed, *n_changed, rows));  // (the new state)
    return DG_OK;
  }
  TRY(splice_edit(e, &w, state_ctx, delta, delta_ctx, keys, n_keys, &w.uctx, true, changed, cap));
  if (const int rc0 = read_counts(e, 6); rc0 != DG_OK) {
    // the join grid could not become resident (another process's persistent kernels) or
    // timed out: nothing of the state is written yet, so re-run the edit on a grid small
    // enough to find room beside other work, as dg_join2_changes does.  Any other failure
    // (a HIP error, a lost publish) is the call's error, its message kept.
    if (!(e->last_err_bits & 3u)) return rc0;
    const int workers = e->join_workers;
    e->join_workers = RETRY_WORKERS;
    HIP_TRY(hipMemsetAsync(e->d_counts + 5, 0, sizeof(u64), e->stream));  // `moved`
    const int rc = splice_edit(e, &w, state_ctx, delta, delta_ctx, keys, n_keys, &w.uctx, true,
                               changed, cap);
    e->join_workers = workers;
    TRY(rc);
    TRY(read_counts(e, 6));
  }
  const bool moved = (u32)e->h_counts[5] != 0;
  const u64 n_e = e->h_counts[0];
  w.uctx.n = e->h_counts[1];
  *n_changed = e->h_counts[2];
  if (*n_changed > cap)
    return fail(DG_E_CAPACITY, "dg_join_delta: %llu changed keys > cap %llu",
                (unsigned long long)*n_changed, (unsigned long long)cap);
  dg_store* out = moved ? spare : state;
  w.sp.out = rows_out_of(out);
  // the copy: into `spare` (scratch until the swap) when rows move, else E's rows in place,
  // guarded by the tree update's error word; then the union context, guarded the same way
  const u32* guard = tree ? e->ticket + 3 : nullptr;
  w.sp.guard = moved ? nullptr : guard;
  auto copy = [&]() -> int {
    HIP_TRY(launch_splice_copy(w.sp, !moved, e->stream));
    HIP_TRY(launch_splice_finish(w.uctx.node, w.uctx.cnt, w.uctx.n, state_ctx->node, state_ctx->cnt,
                                 nullptr, 0, nullptr, nullptr, e->stream, guard));
    return DG_OK;
  };
  dg_store ed = w.ed;  // the keyset's joined rows (scratch, key order)
  ed.n = n_e;
  if (tree) {
    // MerkleMap.put/delete of the changed keys: every changed key is a keyset key, so its
    // old rows are among the taken rows and its new rows among the edit's (both small and
    // cache-resident: no search of the 12.5M-row state)
    u64 dk = 0;
    TRY(tree_update(e, tree, &w.ak, &ed, changed, *n_changed, "dg_join_delta", false, copy, &dk));
    tree->n_keys += dk;
  } else {
    TRY(copy());
    TRY(read_counts(e, 0));
  }
  out->n = old_state.n - w.n_ak + n_e;
  state_ctx->n = w.uctx.n;
  state_ctx->kind = out_kind;
  if (moved) {
    std::swap(*state, *spare);
    *swapped = 1;
  }
  // the changed keys' rows from the edit (a changed key is a keyset key: all of its
  // joined rows are in the edit), not by a search of the state
  if (rows) TRY(take_changed_rows(e, &ed, changed, *n_changed, rows));
  return DG_OK;
}

// dg_join_delta_home: the fused small-delta join (small.hip) with ONE host wait.  States
// of up to SMALL_COPY_TILES splice tiles get the moved-rows copy in the tail launch behind
// the join (merkle.hip small_tail_kernel: with the tree's upsweep and the publish),
// guarded by its `moved` word; a larger state whose rows moved copies after the wait.
constexpr u64 SMALL_COPY_TILES = 64;
static_assert(DIFF_MISMATCH == DG_DIFF_MISMATCH, "deltagpu.h and the diff kernels agree");
static_assert(CS_IN == DG_CONT_HOME_ENTRIES && CS_B == DG_CONT_HOME_BUCKETS && CONT_HOME + CS_HDR <= 24,
              "deltagpu.h's limits; the header fits the publish block");
static_assert(SMALL_O_KEYS == DG_HOME_KEYS &&SMALL_O_ROWS == DG_HOME_ROWS && SMALL_EDIT == DG_HOME_STRIDE &&
                  SMALL_O_CTX == DG_HOME_CTX && SMALL_NODES == DG_HOME_NODES && SMALL_WORDS == DG_HOME_WORDS &&
                  SMALL_FALLBACK == DG_HOME_FALLBACK,
              "the result block is the header's home layout");

int dg_join_delta_home(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                       const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                       dg_store* spare, dg_merkle* tree, uint64_t* home, int* swapped) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (!swapped || !spare || !state || !state_ctx || !home)
    return fail(DG_E_INVAL, "dg_join_delta_home: null argument");
  *swapped = 0;
  home[0] = SMALL_FALLBACK;
  TRY(check_store(state, "dg_join_delta_home state"));
  TRY(check_store(delta, "dg_join_delta_home delta"));
  TRY(check_ctx(state_ctx, "dg_join_delta_home state_ctx"));
  TRY(check_ctx(delta_ctx, "dg_join_delta_home delta_ctx"));
  if (tree) TRY(check_merkle(tree, "dg_join_delta_home tree"));
  if (keys == nullptr && n_keys != 0) return fail(DG_E_INVAL, "dg_join_delta_home: keys NULL with n_keys>0");
  const bool small = n_keys <= SMALL_KEYS && delta->n <= SMALL_DELTA && delta_ctx->n <= SMALL_DCTX &&
                     state_ctx->kind == DG_CTX_VV && state_ctx->n <= SMALL_NODES &&
                     spare->cap >= state->n + delta->n && state_ctx->cap >= 1 &&
                     pair_aligned(state->key, state->val, state->ts, state->node, state->cnt) &&
                     pair_aligned(spare->key, spare->val, spare->ts, spare->node, spare->cnt);
  if (!small) return DG_OK;  // home[0] = SMALL_FALLBACK: the caller takes dg_join_delta_rows
  TRY(set_device(e));
  TRY(settle(e));
  const u64 nk = n_keys, a_tiles = splice_tiles(state->n);
  const bool copy_now = a_tiles <= SMALL_COPY_TILES;
  // scratch: the edit | a_lo | a_off | end | shift | gap | tile_u0 | moved word | result
  const size_t idx = ((nk + 1) * 8 + 255) / 256 * 256;
  const size_t bytes = (SMALL_EDIT * 36 + 5 * 256) + 6 * idx + ((a_tiles + 2) * 8 + 255) / 256 * 256 + 256 +
                       SMALL_WORDS * 8 + 256;
  TRY(ensure_buf(e, &e->sml, &e->sml_cap, bytes));
  char* q = (char*)e->sml;
  dg_store ed = carve_store(q, SMALL_EDIT);
  u64* a_lo = (u64*)q;
  u64* a_off = (u64*)(q + idx);
  u64* end = (u64*)(q + 2 * idx);
  i64* shift = (i64*)(q + 3 * idx);
  i64* gap = (i64*)(q + 4 * idx);
  q += 6 * idx;
  u64* tile_u0 = (u64*)q;
  q += ((a_tiles + 2) * 8 + 255) / 256 * 256;
  u32* moved_word = (u32*)q;
  q += 256;
  u64* res = (u64*)q;
  SmallArgs p{};
  p.a = rows_of(state);
  p.aw = rows_out_of(state);
  p.ca = ctx_of(state_ctx);
  p.ca_node = state_ctx->node;
  p.ca_cnt = state_ctx->cnt;
  p.ca_cap = state_ctx->cap;
  p.d = rows_of(delta);
  p.cd = ctx_of(delta_ctx);
  p.keys = keys;
  p.nk = nk;
  p.e = rows_out_of(&ed);
  p.a_lo = a_lo;
  p.a_off = a_off;
  p.res = res;
  p.has_tree = tree != nullptr;
  if (tree) p.t = merkle_of(tree);  // MerkleMap.put/delete + update_hashes: in the join
  p.splice_here = copy_now;
  p.sp = rows_out_of(spare);
  p.end = end;
  p.shift = shift;
  p.home = home;
  p.d_counts = e->d_counts;
  p.h_pub = e->d_pub;
  p.seq = ++e->pub_seq;
  HIP_TRY(launch_small_delta(p, e->stream));
  if (copy_now) {  // the moved rows' copy into the spare (if they moved: else it returns)
    SmallTailArgs ta{};
    ta.a = rows_of(state);
    ta.out = rows_out_of(spare);
    ta.end = end;
    ta.a_lo = a_lo;
    ta.shift = shift;
    ta.nk = nk;
    ta.tiles = a_tiles;
    ta.res = res;
    ta.d_counts = e->d_counts;
    ta.h_pub = e->d_pub;
    ta.seq = p.seq;
    ta.arrive_all = e->ticket + TAIL_ARRIVE;
    HIP_TRY(launch_small_tail(ta, e->stream));
  }
  TRY(wait_published(e, p.seq));  // the one wait (the result block is in `home` by then)
  SpliceArgs sp{};
  sp.a = rows_of(state);
  sp.keys = keys;
  sp.nk = nk;
  sp.a_lo = a_lo;
  sp.a_off = a_off;
  sp.end = end;
  sp.shift = shift;
  sp.gap = gap;
  sp.tile_u0 = tile_u0;
  sp.moved = moved_word;
  sp.e = rows_of(&ed);
  sp.e.n = SMALL_EDIT;  // a bound: the kernels read the count
  sp.d_ne = res + 4;
  sp.out = rows_out_of(spare);
  sp.run_if = res + 6;  // the rows moved (0 also when the join fell back or failed)
  const u64 flags = home[0];
  if (flags & SMALL_FALLBACK) return DG_OK;  // nothing written: the general path
  if (flags & MERKLE_INPUT_ERR) {
    if (flags & MERKLE_ERR_SHARD) return fail(DG_E_INVAL, "dg_join_delta_home: a key outside the tree's shard");
    return fail(DG_E_CAPACITY, "dg_join_delta_home: a bucket would hold more than 65535 rows (use a deeper tree)");
  }
  const u64 n_e = home[4], n_ak = home[5];
  if (home[6]) {  // rows moved: the state is in `spare` (copied behind the join, or now)
    if (!copy_now) {
      HIP_TRY(launch_splice_index(sp, e->stream));
      HIP_TRY(launch_splice_copy(sp, false, e->stream));
      TRY(read_counts(e, 0));
    }
    const u64 n = state->n - n_ak + n_e;
    std::swap(*state, *spare);
    state->n = n;
    *swapped = 1;
  }
  state_ctx->n = home[3];
  state_ctx->kind = DG_CTX_VV;
  if (tree) tree->n_keys += home[7];
  return DG_OK;
}

static int join_delta_impl(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                           const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                           dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                           uint64_t* n_changed, int* swapped, dg_store* rows, dg_context* ctx_out = nullptr) {
  bool kd_done = false;
  TRY(join_delta_core(e, state, state_ctx, delta, delta_ctx, keys, n_keys, spare, tree, changed, cap, n_changed,
                      swapped, rows, ctx_out, &kd_done));
  if (ctx_out && !kd_done) {  // (the other paths: the context copied after the join)
    ctx_out->n = state_ctx->n;
    ctx_out->kind = state_ctx->kind;
    if (state_ctx->n <= ctx_out->cap && state_ctx->n) {
      HIP_TRY(hipMemcpyAsync(ctx_out->node, state_ctx->node, state_ctx->n * 4, hipMemcpyDefault, e->stream));
      HIP_TRY(hipMemcpyAsync(ctx_out->cnt, state_ctx->cnt, state_ctx->n * 8, hipMemcpyDefault, e->stream));
      HIP_TRY(hipStreamSynchronize(e->stream));
    }
  }
  return DG_OK;
}

int dg_join_delta(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                  const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                  dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                  uint64_t* n_changed, int* swapped) {
  return join_delta_impl(e, state, state_ctx, delta, delta_ctx, keys, n_keys, spare, tree, changed,
                         cap, n_changed, swapped, nullptr);
}

int dg_join_delta_rows(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                       const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                       dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                       uint64_t* n_changed, int* swapped, dg_store* rows) {
  if (!rows) return fail(DG_E_INVAL, "dg_join_delta_rows: null rows");
  return join_delta_impl(e, state, state_ctx, delta, delta_ctx, keys, n_keys, spare, tree, changed,
                         cap, n_changed, swapped, rows);
}

int dg_join_delta_out(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                      const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                      dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                      uint64_t* n_changed, int* swapped, dg_store* rows, dg_context* ctx_out) {
  if (!rows || !ctx_out) return fail(DG_E_INVAL, "dg_join_delta_out: null rows or ctx_out");
  return join_delta_impl(e, state, state_ctx, delta, delta_ctx, keys, n_keys, spare, tree, changed,
                         cap, n_changed, swapped, rows, ctx_out);
}

}  // extern "C"

namespace {

// Two intermediate states (rows + context) for a fold over at most `rows` rows and
// `ctx` context entries, carved from engine scratch that persists across calls.
int fold_buffers(dg_engine* e, u64 rows, u64 ctx, dg_store* st, dg_context* cx) {
  const size_t half = ((rows * 36 + ctx * 12 + 1024) + 255) / 256 * 256;
  TRY(ensure_buf(e, &e->fold, &e->fold_cap, 2 * half));
  for (int w = 0; w < 2; w++) {
    char* p = (char*)e->fold + w * half;
    st[w].key = (uint64_t*)p;
    p += rows * 8;
    st[w].val = (uint64_t*)p;
    p += rows * 8;
    st[w].ts = (int64_t*)p;
    p += rows * 8;
    st[w].cnt = (uint64_t*)p;
    p += rows * 8;
    cx[w].cnt = (uint64_t*)p;
    p += ctx * 8;
    st[w].node = (uint32_t*)p;
    p += rows * 4;
    cx[w].node = (uint32_t*)p;
    st[w].cap = rows;
    cx[w].cap = ctx;
    st[w].n = 0;
    cx[w].n = 0;
    cx[w].kind = DG_CTX_VV;
  }
  return DG_OK;
}

int copy_state(dg_engine* e, const dg_store* s, const dg_context* c, dg_store* out,
               dg_context* out_ctx) {
  if (out->cap < s->n || out_ctx->cap < c->n) return fail(DG_E_CAPACITY, "output capacity too small");
  if (s->n) {
    HIP_TRY(hipMemcpyAsync(out->key, s->key, s->n * 8, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(out->val, s->val, s->n * 8, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(out->ts, s->ts, s->n * 8, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(out->node, s->node, s->n * 4, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(out->cnt, s->cnt, s->n * 8, hipMemcpyDeviceToDevice, e->stream));
  }
  if (c->n) {
    HIP_TRY(hipMemcpyAsync(out_ctx->node, c->node, c->n * 4, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(out_ctx->cnt, c->cnt, c->n * 8, hipMemcpyDeviceToDevice, e->stream));
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  out->n = s->n;
  out_ctx->n = c->n;
  out_ctx->kind = c->kind;
  return DG_OK;
}

// acc <- join(acc, s_i, keys_i) for i = 0..k-1 (acc starts as (state, ctx)); the last
// step writes into out.
int fold_join(dg_engine* e, const dg_store* state, const dg_context* ctx, int k,
              const dg_store* stores, const dg_context* ctxs, const uint64_t* const* keys,
              const uint64_t* n_keys, dg_store* out, dg_context* out_ctx, const char* what) {
  u64 total = state->n, total_ctx = ctx->n;
  for (int s = 0; s < k; s++) {
    TRY(check_store(&stores[s], what));
    TRY(check_ctx(&ctxs[s], what));
    total += stores[s].n;
    total_ctx += ctxs[s].n;
  }
  if (out->cap < total || out_ctx->cap < total_ctx)
    return fail(DG_E_CAPACITY, "%s: output capacity too small (%llu rows, %llu ctx needed)", what,
                (unsigned long long)total, (unsigned long long)total_ctx);
  TRY(set_device(e));
  if (k == 0) return copy_state(e, state, ctx, out, out_ctx);
  dg_store buf[2];
  dg_context bufc[2];
  if (k > 1) TRY(fold_buffers(e, total, total_ctx, buf, bufc));
  dg_store acc = *state;
  dg_context acc_ctx = *ctx;
  for (int s = 0; s < k; s++) {
    dg_store* dst = (s == k - 1) ? out : &buf[s & 1];
    dg_context* dstc = (s == k - 1) ? out_ctx : &bufc[s & 1];
    dst->n = 0;
    const uint64_t* ks = keys ? keys[s] : nullptr;
    const uint64_t nk = (keys && keys[s]) ? n_keys[s] : 0;
    TRY(dg_join2(e, &acc, &acc_ctx, &stores[s], &ctxs[s], ks, nk, dst, dstc));
    acc = *dst;
    acc_ctx = *dstc;
  }
  return DG_OK;
}

// One pass of dg_apply_deltas over k <= KFOLD_MAX_K deltas (kfold.hip).  *stepwise is
// set when this input needs the delta-by-delta fold instead: a context that is not a
// version vector, a node id >= KNT, or a key bucket over its LDS capacity (keys far
// from uniform hashes).  The state and deltas are only read.
int kfold_pass(dg_engine* e, const dg_store* state, const dg_context* ctx, int k,
               const dg_store* deltas, const dg_context* dctxs, const uint64_t* const* keys,
               const uint64_t* n_keys, dg_store* out, dg_context* out_ctx, bool* stepwise) {
  *stepwise = true;
  if (k < 1 || k > KFOLD_MAX_K || ctx->kind != DG_CTX_VV) return DG_OK;
  u64 m_rows = 0, m_keys = 0, allmask = 0, dotsmask = 0, n_dots = 0;
  for (int i = 0; i < k; i++) {
    if (deltas[i].n >= (1ull << 32)) return DG_OK;
    if (dctxs[i].kind == DG_CTX_DOTS) {  // a mutation delta's MapSet context
      dotsmask |= 1ull << i;
      n_dots += dctxs[i].n;
    }
    const bool full = !keys || !keys[i];
    const u64 nk = full ? 0 : n_keys[i];
    if (nk >= (1ull << 32)) return DG_OK;
    if (full) allmask |= 1ull << i;
    m_rows += deltas[i].n;
    m_keys += nk;
  }
  auto ceil_div = [](u64 a, u64 b) { return (a + b - 1) / b; };
  const u64 T0 = std::max<u64>({ceil_div(state->n, KFOLD_MEAN_S), ceil_div(m_rows, KFOLD_MEAN_D),
                                ceil_div(m_keys, KFOLD_MEAN_M),
                                ceil_div(m_rows + m_keys, KFOLD_MEAN_U), 1});
  // a bucket over capacity (key groups far larger than the mean, or keys that are not
  // uniform hashes) is retried once with 8x the buckets
  for (int attempt = 0; attempt < 2; attempt++) {
    const u64 T = T0 << (3 * attempt);
    if (T >= (1ull << 31)) return DG_OK;
    // device scratch: runs | cflat | sstart | dstart | tabC | tabP | flag | dset
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t b_runs = al(k * sizeof(KRun));
    const size_t b_cf = al((k + 1) * sizeof(u64));
    const size_t b_ss = al((T + 1) * 8), b_ds = al((T + 1) * 2 * k * 4), b_tab = al((size_t)k * KNT * 8);
    u64 dset_n = 1024;  // a power of two at least twice the dots: probes stay short
    while (dset_n < 2 * n_dots) dset_n <<= 1;
    const size_t b_dset = dotsmask ? al(dset_n * 8) : 0;
    const size_t bytes = b_runs + b_cf + b_ss + b_ds + 2 * b_tab + 256 + b_dset;
    TRY(ensure_state(e, T + 2));
    TRY(ensure_tmp(e, bytes));
    const size_t hb = b_runs + b_cf;
    if (hb > e->h_stage_cap) {
      HIP_TRY(hipStreamSynchronize(e->stream));
      if (e->h_stage) HIP_TRY(hipHostFree(e->h_stage));
      e->h_stage = nullptr;
      e->h_stage_cap = 0;
      if (hipHostMalloc(&e->h_stage, hb, 0) != hipSuccess)
        return fail(DG_E_NOMEM, "pinned staging of %zu bytes failed", hb);
      e->h_stage_cap = hb;
    }
    KRun* hr = (KRun*)e->h_stage;
    for (int i = 0; i < k; i++) {
      hr[i].rows = rows_of(&deltas[i]);
      const bool full = !keys || !keys[i];
      hr[i].keys = full ? nullptr : keys[i];
      hr[i].n_keys = full ? 0 : n_keys[i];
      hr[i].ctx = ctx_of(&dctxs[i]);
    }
    u64 max_run = 0;  // the fill's slices per run: a multiple of 8, each <= KFOLD_FILL_SLICE
    for (int i = 0; i < k; i++) max_run = std::max<u64>({max_run, deltas[i].n, hr[i].n_keys});
    const u64 fill_p = 8 * std::max<u64>(1, ceil_div(max_run, 8 * KFOLD_FILL_SLICE));
    if (fill_p >= (1ull << 31)) return DG_OK;
    u64* hc = (u64*)((char*)e->h_stage + b_runs);
    hc[0] = 0;
    for (int i = 0; i < k; i++) hc[i + 1] = hc[i] + (((dotsmask >> i) & 1) ? dctxs[i].n : 0);
    char* d = (char*)e->tmp;
    KFoldArgs p{};
    p.s = rows_of(state);
    p.c0 = ctx_of(ctx);
    p.runs = (const KRun*)d;
    p.cflat = (const u64*)(d + b_runs);
    char* d2 = d + b_runs + b_cf;
    p.sstart = (u64*)d2;
    p.dstart = (u32*)(d2 + b_ss);
    p.tabC = (u64*)(d2 + b_ss + b_ds);
    p.tabP = (u64*)(d2 + b_ss + b_ds + b_tab);
    p.flag = (u32*)(d2 + b_ss + b_ds + 2 * b_tab);
    p.dotsmask = dotsmask;
    p.dset = dotsmask ? (u64*)(d2 + b_ss + b_ds + 2 * b_tab + 256) : nullptr;
    p.dset_mask = dset_n - 1;
    p.dset_n = hc[k];
    p.k = k;
    p.allmask = allmask;
    p.T = T;
    p.fill_p = (u32)fill_p;  // the delta runs; the state's starts: kfold_fill_kernel's
                             // trailing workgroups (state_start, one wave per bucket)
    p.out = rows_out_of(out);
    p.out_ctx_node = out_ctx->node;
    p.out_ctx_cnt = out_ctx->cnt;
    p.d_counts = e->d_counts;
    HIP_TRY(hipMemcpyAsync(d, e->h_stage, hb, hipMemcpyHostToDevice, e->stream));
    // start tables (empty runs keep 0), VV tables (absent node = 0) and the flag; the
    // dot set's slots empty (all ones)
    HIP_TRY(hipMemsetAsync(p.sstart, 0, b_ss + b_ds + 2 * b_tab + 256, e->stream));
    if (dotsmask) HIP_TRY(hipMemsetAsync(p.dset, 0xFF, dset_n * 8, e->stream));
    TRY(next_scan(e, &p.scan));
    HIP_TRY(launch_kfold(p, e->stream));
    HIP_TRY(hipMemcpyAsync(&e->h_counts[10], p.flag, sizeof(u32), hipMemcpyDeviceToHost, e->stream));
    TRY(read_counts(e, 2));  // synchronizes; the staging buffer is free again
    u32 flag = 0;
    memcpy(&flag, &e->h_counts[10], sizeof(u32));
    if (flag & KF_PREP_FAIL) return DG_OK;
    if (flag) continue;
    out->n = e->h_counts[0];
    out_ctx->n = e->h_counts[1];
    out_ctx->kind = DG_CTX_VV;
    *stepwise = false;
    return DG_OK;
  }
  return DG_OK;
}

// dg_apply_deltas: passes of up to KFOLD_MAX_K deltas (each a one-pass fold), or the
// delta-by-delta fold when an input needs it.
int apply_deltas(dg_engine* e, const dg_store* state, const dg_context* ctx, int k,
                 const dg_store* deltas, const dg_context* dctxs, const uint64_t* const* keys,
                 const uint64_t* n_keys, dg_store* out, dg_context* out_ctx) {
  if (e->apply_mode == 1 || k == 0)
    return fold_join(e, state, ctx, k, deltas, dctxs, keys, n_keys, out, out_ctx,
                     "dg_apply_deltas");
  u64 total = state->n, total_ctx = ctx->n;
  for (int s = 0; s < k; s++) {
    TRY(check_store(&deltas[s], "dg_apply_deltas delta"));
    TRY(check_ctx(&dctxs[s], "dg_apply_deltas delta ctx"));
    total += deltas[s].n;
    total_ctx += dctxs[s].n;
  }
  if (out->cap < total || out_ctx->cap < total_ctx)
    return fail(DG_E_CAPACITY, "dg_apply_deltas: output capacity too small (%llu rows, %llu ctx needed)",
                (unsigned long long)total, (unsigned long long)total_ctx);
  if (total && (!out->key || !out->val || !out->ts || !out->node || !out->cnt))
    return fail(DG_E_INVAL, "dg_apply_deltas: null output column");
  TRY(set_device(e));
  const int passes = (k + KFOLD_MAX_K - 1) / KFOLD_MAX_K;
  dg_store buf[2];
  dg_context bufc[2];
  if (passes > 1) TRY(fold_buffers(e, total, total_ctx, buf, bufc));
  dg_store acc = *state;
  dg_context acc_ctx = *ctx;
  for (int q = 0; q < passes; q++) {
    const int i0 = q * KFOLD_MAX_K, kq = std::min(KFOLD_MAX_K, k - i0);
    dg_store* dst = (q == passes - 1) ? out : &buf[q & 1];
    dg_context* dstc = (q == passes - 1) ? out_ctx : &bufc[q & 1];
    bool stepwise = false;
    TRY(kfold_pass(e, &acc, &acc_ctx, kq, deltas + i0, dctxs + i0, keys ? keys + i0 : nullptr,
                   n_keys ? n_keys + i0 : nullptr, dst, dstc, &stepwise));
    if (stepwise && e->apply_mode == 2)
      return fail(DG_E_INVAL, "dg_apply_deltas: one-pass fold not applicable to this input");
    if (stepwise)  // from the original state: fold_join reuses the ping-pong buffers
      return fold_join(e, state, ctx, k, deltas, dctxs, keys, n_keys, out, out_ctx,
                       "dg_apply_deltas");
    acc = *dst;
    acc_ctx = *dstc;
  }
  return DG_OK;
}

}  // namespace

extern "C" {

int dg_joink(dg_engine* e, int k, const dg_store* stores, const dg_context* ctxs, dg_store* out,
             dg_context* out_ctx) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (k <= 0 || !stores || !ctxs || !out || !out_ctx) return fail(DG_E_INVAL, "dg_joink: bad args");
  TRY(check_store(&stores[0], "dg_joink store"));
  TRY(check_ctx(&ctxs[0], "dg_joink ctx"));
  TRY(settle(e));
  return fold_join(e, &stores[0], &ctxs[0], k - 1, stores + 1, ctxs + 1, nullptr, nullptr, out,
                   out_ctx, "dg_joink");
}

int dg_apply_deltas(dg_engine* e, const dg_store* state, const dg_context* ctx, int k,
                    const dg_store* deltas, const dg_context* dctxs,
                    const uint64_t* const* keys, const uint64_t* n_keys, dg_store* out,
                    dg_context* out_ctx) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (k < 0 || (k > 0 && (!deltas || !dctxs)) || !out || !out_ctx)
    return fail(DG_E_INVAL, "dg_apply_deltas: bad args");
  TRY(check_store(state, "dg_apply_deltas state"));
  TRY(check_ctx(ctx, "dg_apply_deltas ctx"));
  if (keys && !n_keys) return fail(DG_E_INVAL, "dg_apply_deltas: keys without n_keys");
  TRY(settle(e));
  return apply_deltas(e, state, ctx, k, deltas, dctxs, keys, n_keys, out, out_ctx);
}

int dg_take_keys(dg_engine* e, const dg_store* s, const uint64_t* keys, uint64_t n_keys,
                 dg_store* out) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_store(s, "dg_take_keys"));
  if (!out || (n_keys && !keys)) return fail(DG_E_INVAL, "dg_take_keys: null argument");
  if (out->cap && (!out->key || !out->val || !out->ts || !out->node || !out->cnt))
    return fail(DG_E_INVAL, "dg_take_keys: null output column");
  TRY(set_device(e));
  TRY(settle(e));
  TRY(ensure_state(e, take_tiles(n_keys) + 1));
  Scan sc;
  TRY(next_scan(e, &sc));
  HIP_TRY(launch_take_keys(rows_of(s), keys, n_keys, rows_out_of(out), out->cap, sc, e->d_counts,
                           e->stream));
  TRY(read_counts(e, 1));
  out->n = e->h_counts[0];
  if (out->n > out->cap)
    return fail(DG_E_CAPACITY, "dg_take_keys: %llu rows > cap %llu", (unsigned long long)out->n,
                (unsigned long long)out->cap);
  return DG_OK;
}

static int mutate_batch_impl(dg_engine* e, const dg_store* state, const dg_context* ctx, uint32_t node,
                             uint64_t m, const uint8_t* kind, const uint64_t* key, const uint64_t* val,
                             const int64_t* ts, const uint64_t* add_rank, uint64_t n_adds, dg_store* delta,
                             dg_context* delta_dots, uint64_t* keys_out, uint64_t keys_cap,
                             uint64_t* n_keys_out, bool sync) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_store(state, "dg_mutate_batch state"));
  TRY(check_ctx(ctx, "dg_mutate_batch ctx"));
  if (ctx->kind != DG_CTX_VV)
    return fail(DG_E_INVAL, "dg_mutate_batch: the state's context must be a version vector "
                            "(compress_dots/1 it first)");
  if (!delta || !delta_dots || !n_keys_out || (m && (!kind || !key || !val || !ts || !add_rank)))
    return fail(DG_E_INVAL, "dg_mutate_batch: null argument");
  if (n_adds > m) return fail(DG_E_INVAL, "dg_mutate_batch: n_adds > m");
  TRY(set_device(e));
  TRY(settle(e));
  const u64 nt = mutate_tiles(m);
  TRY(ensure_state(e, 6 * nt + 2));  // raw per-tile counts and offsets
  HIP_TRY(hipMemsetAsync(e->ticket + 3, 0, sizeof(u32), e->stream));
  u32* err = e->ticket + 3;
  HIP_TRY(launch_mutate_count(rows_of(state), ctx_of(ctx), node, kind, key, val, ts, add_rank, m,
                              e->state, e->d_counts, err, e->ticket + MUT_ARRIVE, e->stream));
  TRY(read_counts(e, 3));  // (the counts and the order flag, err = ticket[3], in one wait)
  const u64 n_keys = e->h_counts[0], n_rows = e->h_counts[1], n_sdots = e->h_counts[2];
  if (e->h_ticket[3] & 1u) return fail(DG_E_ORDER, "dg_mutate_batch: ops are not sorted by key");
  const u64 n_dots = n_sdots + n_adds;
  if (keys_cap < n_keys || delta->cap < n_rows || delta_dots->cap < n_dots)
    return fail(DG_E_CAPACITY,
                "dg_mutate_batch: needs %llu keys, %llu delta rows, %llu context dots",
                (unsigned long long)n_keys, (unsigned long long)n_rows, (unsigned long long)n_dots);
  if ((n_keys && !keys_out) || (n_rows && (!delta->key || !delta->val || !delta->ts ||
                                           !delta->node || !delta->cnt)) ||
      (n_dots && (!delta_dots->node || !delta_dots->cnt)))
    return fail(DG_E_INVAL, "dg_mutate_batch: null output column");
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t sort_b = al(mutate_sort_tmp_bytes(n_dots)), n4 = al(n_dots * 4), n8 = al(n_dots * 8);
  TRY(ensure_tmp(e, 2 * (n4 + n8) + sort_b + 256));
  char* t = (char*)e->tmp;
  u32* dnode = (u32*)t;
  u64* dcnt = (u64*)(t + n4);
  u32* tnode = (u32*)(t + n4 + n8);
  u64* tcnt = (u64*)(t + 2 * n4 + n8);
  void* sort_tmp = t + 2 * (n4 + n8);
  HIP_TRY(launch_mutate_write(rows_of(state), ctx_of(ctx), node, kind, key, val, ts, add_rank, m,
                              e->state, keys_out, rows_out_of(delta), dnode, dcnt, err, e->stream));
  HIP_TRY(launch_mutate_dots(ctx_of(ctx), node, n_adds, n_sdots, dnode, dcnt, tnode, tcnt, sort_tmp,
                             sort_b, delta_dots->node, delta_dots->cnt, e->stream));
  if (sync) HIP_TRY(hipStreamSynchronize(e->stream));
  delta->n = n_rows;
  delta_dots->n = n_dots;
  delta_dots->kind = DG_CTX_DOTS;
  *n_keys_out = n_keys;
  return DG_OK;
}

int dg_mutate_batch(dg_engine* e, const dg_store* state, const dg_context* ctx, uint32_t node,
                    uint64_t m, const uint8_t* kind, const uint64_t* key, const uint64_t* val,
                    const int64_t* ts, const uint64_t* add_rank, uint64_t n_adds, dg_store* delta,
                    dg_context* delta_dots, uint64_t* keys_out, uint64_t keys_cap,
                    uint64_t* n_keys_out) {
  return mutate_batch_impl(e, state, ctx, node, m, kind, key, val, ts, add_rank, n_adds, delta, delta_dots,
                           keys_out, keys_cap, n_keys_out, true);
}

int dg_mutate_batch_async(dg_engine* e, const dg_store* state, const dg_context* ctx, uint32_t node,
                          uint64_t m, const uint8_t* kind, const uint64_t* key, const uint64_t* val,
                          const int64_t* ts, const uint64_t* add_rank, uint64_t n_adds, dg_store* delta,
                          dg_context* delta_dots, uint64_t* keys_out, uint64_t keys_cap,
                          uint64_t* n_keys_out) {
  return mutate_batch_impl(e, state, ctx, node, m, kind, key, val, ts, add_rank, n_adds, delta, delta_dots,
                           keys_out, keys_cap, n_keys_out, false);
}

int dg_context_union(dg_engine* e, const dg_context* a, const dg_context* b, dg_context* out) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_ctx(a, "dg_context_union a"));
  TRY(check_ctx(b, "dg_context_union b"));
  if (!out) return fail(DG_E_INVAL, "dg_context_union: null out");
  if (out->cap < a->n + b->n) return fail(DG_E_CAPACITY, "dg_context_union: out cap too small");
  TRY(set_device(e));
  TRY(settle(e));
  TRY(ensure_tmp(e, ctx_union_tmp_bytes(a->n, b->n)));
  HIP_TRY(launch_ctx_union(ctx_of(a), ctx_of(b), out->node, out->cnt, e->d_counts + 1, e->tmp,
                           e->stream));
  TRY(read_counts(e, 2));
  out->n = e->h_counts[1];
  out->kind = (a->kind == DG_CTX_DOTS && b->kind == DG_CTX_DOTS) ? DG_CTX_DOTS : DG_CTX_VV;
  return DG_OK;
}

int dg_compress_dots(dg_engine* e, const dg_context* dots, dg_context* out_vv) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_ctx(dots, "dg_compress_dots"));
  if (dots->kind != DG_CTX_DOTS)
    return fail(DG_E_CLAUSE,
                "no function clause matching in DeltaCrdt.AWLWWMap.Dots.compress/1 "
                "(context is already a version vector; aw_lww_map.ex:13)");
  dg_context empty;
  memset(&empty, 0, sizeof empty);
  empty.kind = DG_CTX_VV;
  return dg_context_union(e, &empty, dots, out_vv);
}

int dg_read_lww(dg_engine* e, const dg_store* s, const uint64_t* keys, uint64_t n_keys,
                uint64_t* out_key, uint64_t* out_val, uint64_t cap, uint64_t* n_out) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_store(s, "dg_read_lww"));
  if (!n_out || (s->n && (!out_key || !out_val))) return fail(DG_E_INVAL, "dg_read_lww: null output");
  if (keys == nullptr && n_keys != 0) return fail(DG_E_INVAL, "dg_read_lww: keys NULL with n_keys>0");
  u64 need = keys ? std::min<u64>(n_keys, s->n) : s->n;
  if (cap < need)
    return fail(DG_E_CAPACITY, "dg_read_lww: cap %llu < %llu", (unsigned long long)cap,
                (unsigned long long)need);
  TRY(set_device(e));
  TRY(settle(e));
  TRY(ensure_state(e, 2 * seg_tiles(s->n) + 2));  // raw per-tile counts and offsets
  HIP_TRY(launch_read_lww(rows_of(s), keys, keys ? n_keys : 0, out_key, out_val, e->state,
                          e->d_counts, e->stream));
  TRY(read_counts(e, 1));
  *n_out = e->h_counts[0];
  return DG_OK;
}

}  // extern "C"

namespace {

MerkleT merkle_of(const dg_merkle* t) {
  MerkleT m;
  m.depth = t->depth;
  m.sb = t->shard_bits;
  m.shard = t->shard;
  m.nodes = t->nodes;
  m.counts = t->counts;
  m.th = TermH{};
  if (t->terms) {
    m.th.nh = t->terms->node_hash;
    m.th.nn = t->terms->node_hash ? t->terms->n_nodes : 0;
    m.th.vid = t->terms->val_id;
    m.th.vh = t->terms->val_hash;
    m.th.nv = (t->terms->val_id && t->terms->val_hash) ? t->terms->n_vals : 0;
    m.th.on = 1;
  }
  m.starts = t->starts;
  return m;
}

int check_merkle(const dg_merkle* t, const char* what) {
  if (!t || !t->nodes) return fail(DG_E_INVAL, "%s: null tree", what);
  if (!t->counts || ((uintptr_t)t->counts & 15))
    return fail(DG_E_INVAL, "%s: the tree's counts must be a 16-byte aligned device array", what);
  if (t->depth < 1 || t->depth > 28) return fail(DG_E_INVAL, "%s: depth %u not in 1..28", what, t->depth);
  if (t->shard_bits > 16 || t->depth + t->shard_bits > 44)
    return fail(DG_E_INVAL, "%s: shard_bits %u (depth %u)", what, t->shard_bits, t->depth);
  if (t->shard_bits ? (t->shard >> t->shard_bits) != 0 : t->shard != 0)
    return fail(DG_E_INVAL, "%s: shard %llu >= 2^%u", what, (unsigned long long)t->shard, t->shard_bits);
  return DG_OK;
}

int same_tree_shape(const dg_merkle* a, const dg_merkle* b, const char* what) {
  if (a->depth != b->depth || a->shard_bits != b->shard_bits || a->shard != b->shard)
    return fail(DG_E_INVAL, "%s: trees of different shape (depth %u/%u, shard %llu/%llu)", what,
                a->depth, b->depth, (unsigned long long)a->shard, (unsigned long long)b->shard);
  return DG_OK;
}

// The input-error word (ticket[3]) after a synchronizing read; bit 1: key outside shard,
// bit 2: a bucket over 65535 rows.  (reads the ticket words of the read_counts before it)
int input_error(dg_engine* e, const char* what) {
  if (e->h_ticket[3] & 2u) return fail(DG_E_INVAL, "%s: a key outside the tree's shard", what);
  if (e->h_ticket[3] & 4u)
    return fail(DG_E_CAPACITY, "%s: a bucket holds more than 65535 rows (use a deeper tree)", what);
  return DG_OK;
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

// The build's launch, shared by the synchronous call, the asynchronous one and the replay.
int merkle_build_enqueue(dg_engine* e, const dg_store* s, dg_merkle* t, uint64_t* d_n_keys) {
  TRY(check_store(s, "dg_merkle_build"));
  TRY(check_merkle(t, "dg_merkle_build"));
  if (!d_n_keys) return fail(DG_E_INVAL, "dg_merkle_build: null d_n_keys");
  TRY(set_device(e));
  TRY(ensure_tmp(e, merkle_ctr_words(t->depth) * sizeof(u32)));
  HIP_TRY(hipMemsetAsync(e->ticket + 3, 0, sizeof(u32), e->stream));
  HIP_TRY(launch_merkle_build(rows_of(s), merkle_of(t), d_n_keys, e->ticket + MERKLE_ARRIVE,
                              (u64*)e->tmp, e->ticket + 3, e->stream));
  return DG_OK;
}

}  // namespace

extern "C" {

int dg_merkle_build_async(dg_engine* e, const dg_store* s, dg_merkle* t, uint64_t* d_n_keys) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (e->pending.size() >= MAX_PENDING) TRY(dg_engine_sync(e));
  TRY(merkle_build_enqueue(e, s, t, d_n_keys));
  dg_engine::Pending q{};
  q.kind = 1;
  q.a = *s;
  q.t = *t;
  q.tp = t;
  q.d_counts = d_n_keys;
  e->pending.push_back(q);
  return DG_OK;
}

int dg_merkle_build(dg_engine* e, const dg_store* s, dg_merkle* t) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(settle(e));
  TRY(merkle_build_enqueue(e, s, t, e->d_counts));  // not logged: it is settled right here
  TRY(read_counts(e, 1));
  TRY(input_error(e, "dg_merkle_build"));
  t->n_keys = e->h_counts[0];
  return DG_OK;
}

int dg_merkle_update(dg_engine* e, dg_merkle* t, const dg_store* old_s, const dg_store* new_s,
                     const uint64_t* keys, uint64_t n_keys) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_merkle(t, "dg_merkle_update"));
  TRY(check_store(old_s, "dg_merkle_update old"));
  TRY(check_store(new_s, "dg_merkle_update new"));
  if (n_keys && !keys) return fail(DG_E_INVAL, "dg_merkle_update: null keys");
  TRY(set_device(e));
  TRY(settle(e));
  return tree_update(e, t, old_s, new_s, keys, n_keys, "dg_merkle_update");
}

int dg_merkle_diff(dg_engine* e, const dg_merkle* a, const dg_store* sa, const dg_merkle* b,
                   const dg_store* sb, uint64_t* out_keys, uint64_t cap, uint64_t* n_out,
                   uint64_t* n_total) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_merkle(a, "dg_merkle_diff a"));
  TRY(check_merkle(b, "dg_merkle_diff b"));
  TRY(same_tree_shape(a, b, "dg_merkle_diff"));
  TRY(check_store(sa, "dg_merkle_diff sa"));
  TRY(check_store(sb, "dg_merkle_diff sb"));
  if (!n_out) return fail(DG_E_INVAL, "dg_merkle_diff: null n_out");
  if (cap && !out_keys) return fail(DG_E_INVAL, "dg_merkle_diff: null out_keys");
  TRY(set_device(e));
  TRY(settle(e));
  TRY(ensure_tmp(e, diff_scratch_words(a->depth, sa->n, sb->n) * sizeof(u64)));
  TRY(ensure_diff_bsum(e, diff_groups(a->depth)));
  HIP_TRY(enqueue_merkle_diff(e, a, sa, b, sb, out_keys, cap, e->d_counts));
  TRY(read_counts(e, 1));
  const u64 total = e->h_counts[0];
  if (total >= DIFF_MISMATCH) {
    *n_out = 0;
    if (n_total) *n_total = 0;
    return fail(DG_E_INVAL, "dg_merkle_diff: a tree counts more rows than its store holds "
                            "(the store is not the one the tree was built / updated against)");
  }
  *n_out = std::min<u64>(total, cap);
  if (n_total) *n_total = total;
  return DG_OK;
}

int dg_merkle_diff_async(dg_engine* e, const dg_merkle* a, const dg_store* sa, const dg_merkle* b,
                         const dg_store* sb, uint64_t* out_keys, uint64_t cap, uint64_t* d_total) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_merkle(a, "dg_merkle_diff_async a"));
  TRY(check_merkle(b, "dg_merkle_diff_async b"));
  TRY(same_tree_shape(a, b, "dg_merkle_diff_async"));
  TRY(check_store(sa, "dg_merkle_diff_async sa"));
  TRY(check_store(sb, "dg_merkle_diff_async sb"));
  if (!d_total) return fail(DG_E_INVAL, "dg_merkle_diff_async: null d_total");
  if (cap && !out_keys) return fail(DG_E_INVAL, "dg_merkle_diff_async: null out_keys");
  TRY(set_device(e));
  TRY(settle(e));  // (a logged join that aborted is replayed before its output is read)
  TRY(ensure_tmp(e, diff_scratch_words(a->depth, sa->n, sb->n) * sizeof(u64)));
  TRY(ensure_diff_bsum(e, diff_groups(a->depth)));
  HIP_TRY(enqueue_merkle_diff(e, a, sa, b, sb, out_keys, cap, d_total));
  return DG_OK;
}

int dg_merkle_prepare(dg_engine* e, const dg_merkle* t, uint32_t levels, dg_merkle_cont* out) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_merkle(t, "dg_merkle_prepare"));
  if (!out || levels < 1) return fail(DG_E_INVAL, "dg_merkle_prepare: bad arguments");
  const u32 L = std::min<u32>(levels, t->depth);
  const u64 n = 1ull << L;
  out->level = L;
  out->n = n;
  out->n_buckets = 0;
  if (out->cap < n || !out->pos || !out->hash)
    return fail(DG_E_CAPACITY, "dg_merkle_prepare: %llu entries needed", (unsigned long long)n);
  TRY(set_device(e));
  TRY(settle(e));
  HIP_TRY(launch_cont_prepare(merkle_of(t), L, out->pos, out->hash, e->stream));
  return sync_words(e);
}

int dg_merkle_continue(dg_engine* e, const dg_merkle* t, const dg_store* s, const dg_merkle_cont* in,
                       uint32_t levels, dg_merkle_cont* out, uint64_t* keys, uint64_t cap,
                       uint64_t* n_keys, uint64_t* n_total, int* status) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_merkle(t, "dg_merkle_continue"));
  TRY(check_store(s, "dg_merkle_continue"));
  if (!in || !status || !n_keys || levels < 1 || (cap && !keys))
    return fail(DG_E_INVAL, "dg_merkle_continue: bad arguments");
  if (in->n && (!in->pos || !in->hash)) return fail(DG_E_INVAL, "dg_merkle_continue: null input");
  *n_keys = 0;
  if (n_total) *n_total = 0;
  *status = 0;
  TRY(set_device(e));
  TRY(settle(e));
  const u32 depth = t->depth;
  const MerkleT m = merkle_of(t);
  if (in->level == depth + 1) {  // leaf form: the keys
    if (in->n_buckets && !in->bucket) return fail(DG_E_INVAL, "dg_merkle_continue: null buckets");
    TRY(ensure_state(e, 2 * cont_tiles(in->n_buckets) + 2));
    HIP_TRY(launch_leafdiff(m, rows_of(s), in->bucket, in->n_buckets, in->pos, in->hash, in->n, keys,
                            cap, e->state, e->d_counts, e->stream));
    TRY(read_counts(e, 1));
    const u64 total = e->h_counts[0];
    *n_keys = std::min<u64>(total, cap);
    if (n_total) *n_total = total;
    return DG_OK;
  }
  if (in->level > depth) return fail(DG_E_INVAL, "dg_merkle_continue: level %u > depth %u", in->level, depth);
  if (!out) return fail(DG_E_INVAL, "dg_merkle_continue: null out");
  const u32 L = in->level;
  TRY(ensure_state(e, 2 * cont_tiles(in->n) + 2));
  TRY(ensure_tmp(e, std::max<u64>(in->n, 1) * sizeof(u64)));
  u64* dpos = (u64*)e->tmp;
  HIP_TRY(launch_cont_compare(m, L, in->pos, in->hash, in->n, e->state, dpos, e->d_counts, e->stream));
  TRY(read_counts(e, 1));
  const u64 nd = e->h_counts[0];
  if (nd == 0) return DG_OK;  // {:ok, []}
  if (L < depth) {
    const u32 k = std::min<u32>(levels, depth - L);
    const u64 need = nd << k;
    out->level = L + k;
    out->n = need;
    out->n_buckets = 0;
    if (out->cap < need || !out->pos || !out->hash)
      return fail(DG_E_CAPACITY, "dg_merkle_continue: %llu entries needed", (unsigned long long)need);
    HIP_TRY(launch_cont_expand(m, L, k, dpos, nd, out->pos, out->hash, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    *status = 1;
    return DG_OK;
  }
  // the differing buckets -> leaf form
  out->level = depth + 1;
  out->n_buckets = nd;
  if (out->cap_buckets < nd || !out->bucket)
    return fail(DG_E_CAPACITY, "dg_merkle_continue: %llu buckets needed", (unsigned long long)nd);
  HIP_TRY(hipMemcpyAsync(out->bucket, dpos, nd * sizeof(u64), hipMemcpyDeviceToDevice, e->stream));
  TRY(ensure_state(e, 2 * cont_tiles(nd) + 2));
  HIP_TRY(launch_leaves_count(m, rows_of(s), out->bucket, nd, e->state, e->d_counts, e->stream));
  TRY(read_counts(e, 1));
  const u64 np = e->h_counts[0];
  out->n = np;
  if (out->cap < np || (np && (!out->pos || !out->hash)))
    return fail(DG_E_CAPACITY, "dg_merkle_continue: %llu leaf pairs needed", (unsigned long long)np);
  HIP_TRY(launch_leaves_write(m, rows_of(s), out->bucket, nd, e->state, out->pos, out->hash, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  *status = 1;
  return DG_OK;
}

int dg_merkle_continue_home(dg_engine* e, const dg_merkle* t, const dg_store* s, const dg_merkle_cont* in,
                            uint32_t levels, uint64_t max, dg_merkle_cont* out, uint64_t* keys, uint64_t cap,
                            uint64_t* n_keys, uint64_t* n_total, int* status) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_merkle(t, "dg_merkle_continue_home"));
  TRY(check_store(s, "dg_merkle_continue_home"));
  if (!in || !status || !n_keys || levels < 1 || (cap && !keys))
    return fail(DG_E_INVAL, "dg_merkle_continue_home: bad arguments");
  if (in->n && (!in->pos || !in->hash)) return fail(DG_E_INVAL, "dg_merkle_continue_home: null input");
  const u32 depth = t->depth;
  const bool leaf = in->level == depth + 1;
  if (in->level > depth + 1) return fail(DG_E_INVAL, "dg_merkle_continue_home: level %u > depth %u", in->level, depth);
  if (leaf && in->n_buckets && !in->bucket) return fail(DG_E_INVAL, "dg_merkle_continue_home: null buckets");
  *n_keys = 0;
  if (n_total) *n_total = 0;
  *status = DG_CONT_DECLINED;
  if (in->n > CS_IN || (leaf && in->n_buckets > CS_B)) return DG_OK;  // the general path
  *status = 0;
  if (leaf ? in->n_buckets == 0 : in->n == 0) return DG_OK;  // {:ok, []}
  if (!leaf && !out) return fail(DG_E_INVAL, "dg_merkle_continue_home: null out");
  TRY(set_device(e));
  TRY(settle(e));
  ContSmallArgs a{};
  a.t = merkle_of(t);
  a.s = rows_of(s);
  a.level = in->level;
  a.levels = levels;
  a.max = max;
  a.ipos = in->pos;
  a.ihash = in->hash;
  a.ibucket = leaf ? in->bucket : nullptr;
  a.n = in->n;
  a.nb = leaf ? in->n_buckets : 0;
  if (out) {
    a.opos = out->pos;
    a.ohash = out->hash;
    a.obucket = out->bucket;
    a.ocap = out->pos && out->hash ? out->cap : 0;
    a.ocap_b = out->bucket ? out->cap_buckets : 0;
  }
  a.keys = keys;
  a.kcap = cap;
  a.home = e->d_pub + CONT_HOME;
  a.d_counts = e->d_counts;
  a.h_pub = e->d_pub;
  a.seq = ++e->pub_seq;
  HIP_TRY(launch_cont_small(a, e->stream));
  TRY(wait_published(e, a.seq));
  u64 h[CS_HDR];
  memcpy(h, (const void*)(e->h_pub + CONT_HOME), sizeof h);
  if (h[0] == CS_BAD)
    return fail(DG_E_INVAL, "dg_merkle_continue_home: a position or bucket outside the tree");
  if (h[0] == CS_CAP) {
    out->level = (u32)h[3];
    out->n = h[4];
    out->n_buckets = h[5];
    *status = 0;
    return fail(DG_E_CAPACITY, "dg_merkle_continue_home: %llu entries / %llu buckets needed",
                (unsigned long long)h[4], (unsigned long long)h[5]);
  }
  if (h[0] == CS_OK) {
    *n_keys = std::min<u64>(h[1], cap);
    if (n_total) *n_total = h[1];
    return DG_OK;
  }
  out->level = (u32)h[3];
  out->n = h[1];
  out->n_buckets = h[0] == CS_LEAF ? h[2] : 0;
  *status = 1;
  return DG_OK;
}

int dg_merkle_truncate(dg_engine* e, const dg_merkle* t, dg_merkle_cont* cont, uint64_t max) {
  if (!e || !cont) return fail(DG_E_INVAL, "dg_merkle_truncate: null argument");
  TRY(check_merkle(t, "dg_merkle_truncate"));
  if (cont->n_buckets == 0 || cont->bucket == nullptr) {  // node form (or an empty leaf form)
    cont->n = std::min<u64>(cont->n, max);
    return DG_OK;
  }
  if (cont->n_buckets <= max) return DG_OK;
  // leaf form: the pairs of the first `max` buckets are those whose key sorts before
  // the first pair of bucket[max]; pairs carry keys, buckets carry bucket numbers, so
  // count the pairs of the dropped buckets by their bucket's first pair
  TRY(set_device(e));
  TRY(settle(e));
  TRY(ensure_state(e, 2));
  HIP_TRY(launch_pairs_before_bucket(merkle_of(t), cont->pos, cont->n, cont->bucket + max,
                                     e->d_counts, e->stream));
  TRY(read_counts(e, 1));
  cont->n = e->h_counts[0];
  cont->n_buckets = max;
  return DG_OK;
}

uint64_t dg_merkle_chunks(uint32_t depth) { return merkle_chunks(depth); }

int dg_merkle_fold_roots(const uint64_t* roots, uint32_t shard_bits, uint64_t* root) {
  if (!roots || !root || shard_bits > 16) return fail(DG_E_INVAL, "dg_merkle_fold_roots: bad arguments");
  std::vector<u64> lvl(roots, roots + (1ull << shard_bits));
  while (lvl.size() > 1) {
    std::vector<u64> up(lvl.size() / 2);
    for (size_t i = 0; i < up.size(); i++) up[i] = node_hash(lvl[2 * i], lvl[2 * i + 1]);
    lvl.swap(up);
  }
  *root = lvl[0];
  return DG_OK;
}

int dg_remap_values(dg_engine* e, dg_store* s, const uint64_t* old_ids, const uint64_t* new_ids,
                    uint64_t n_ids) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_store(s, "dg_remap_values"));
  if (n_ids && (!old_ids || !new_ids)) return fail(DG_E_INVAL, "dg_remap_values: null id table");
  if (s->n == 0) return DG_OK;
  TRY(set_device(e));
  TRY(settle(e));
  HIP_TRY(hipMemsetAsync(e->ticket + 3, 0, sizeof(u32), e->stream));
  HIP_TRY(launch_remap_values(s->val, s->n, old_ids, new_ids, n_ids, e->ticket + 3, e->stream));
  TRY(sync_words(e));
  if (e->h_ticket[3]) return fail(DG_E_INVAL, "dg_remap_values: a row's value id is not in old_ids");
  return DG_OK;
}

int dg_sort_store(dg_engine* e, const dg_store* in, dg_store* out) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_store(in, "dg_sort_store"));
  if (!out) return fail(DG_E_INVAL, "dg_sort_store: null out");
  if (out->cap < in->n)
    return fail(DG_E_CAPACITY, "dg_sort_store: out cap %llu < %llu rows", (unsigned long long)out->cap,
                (unsigned long long)in->n);
  if (in->n && (!out->key || !out->val || !out->ts || !out->node || !out->cnt))
    return fail(DG_E_INVAL, "dg_sort_store: null output column");
  if (in->n >= (1ull << 32)) return fail(DG_E_INVAL, "dg_sort_store: more than 2^32 - 1 rows");
  TRY(set_device(e));
  TRY(settle(e));
  TRY(ensure_tmp(e, sort_tmp_bytes(in->n)));
  TRY(ensure_stage(e, 8 * 256 * sizeof(u32)));
  HIP_TRY(launch_sort_store(rows_of(in), rows_out_of(out), e->tmp, (u32*)e->h_stage, e->d_counts,
                            e->stream));
  TRY(read_counts(e, 1));
  out->n = e->h_counts[0];
  return DG_OK;
}

int dg_sort_context(dg_engine* e, const dg_context* in, dg_context* out) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  TRY(check_ctx(in, "dg_sort_context"));
  if (!out) return fail(DG_E_INVAL, "dg_sort_context: null out");
  if (out->cap < in->n) return fail(DG_E_CAPACITY, "dg_sort_context: out cap too small");
  if (in->n && (!out->node || !out->cnt)) return fail(DG_E_INVAL, "dg_sort_context: null output");
  if (in->n >= (1ull << 32)) return fail(DG_E_INVAL, "dg_sort_context: more than 2^32 - 1 entries");
  TRY(set_device(e));
  TRY(settle(e));
  TRY(ensure_tmp(e, sort_tmp_bytes(in->n)));
  TRY(ensure_stage(e, 8 * 256 * sizeof(u32)));
  HIP_TRY(launch_sort_context(in->kind, in->node, in->cnt, in->n, out->node, out->cnt, e->tmp,
                              (u32*)e->h_stage, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  out->n = in->n;
  out->kind = in->kind;
  return DG_OK;
}

// ---- device buffers
int dg_buffer_alloc(dg_engine* e, uint64_t bytes, void** p) {
  if (!e || !p) return fail(DG_E_INVAL, "dg_buffer_alloc: null argument");
  *p = nullptr;
  TRY(set_device(e));
  if (bytes == 0) return DG_OK;
  if (hipMalloc(p, bytes) != hipSuccess) {
    *p = nullptr;
    return fail(DG_E_NOMEM, "hipMalloc of %llu bytes failed", (unsigned long long)bytes);
  }
  return DG_OK;
}

int dg_buffer_free(dg_engine* e, void* p) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (!p) return DG_OK;
  TRY(set_device(e));
  HIP_TRY(hipStreamSynchronize(e->stream));  // no kernel of this engine still uses it
  HIP_TRY(hipFree(p));
  return DG_OK;
}

int dg_copy_to_device(dg_engine* e, void* dst, const void* src, uint64_t bytes) {
  if (!e || (bytes && (!dst || !src))) return fail(DG_E_INVAL, "dg_copy_to_device: null argument");
  if (!bytes) return DG_OK;
  TRY(set_device(e));
  // (hipMemcpyDefault: the source may be device memory too -- a device-to-device copy)
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return DG_OK;
}

int dg_copy_to_host(dg_engine* e, void* dst, const void* src, uint64_t bytes) {
  if (!e || (bytes && (!dst || !src))) return fail(DG_E_INVAL, "dg_copy_to_host: null argument");
  if (!bytes) return DG_OK;
  TRY(set_device(e));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return DG_OK;
}

int dg_copy_async(dg_engine* e, void* dst, const void* src, uint64_t bytes) {
  if (!e || (bytes && (!dst || !src))) return fail(DG_E_INVAL, "dg_copy_async: null argument");
  if (!bytes) return DG_OK;
  TRY(set_device(e));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, e->stream));
  return DG_OK;
}

int dg_host_alloc(dg_engine* e, uint64_t bytes, void** p) {
  if (!e || !p) return fail(DG_E_INVAL, "dg_host_alloc: null argument");
  *p = nullptr;
  TRY(set_device(e));
  if (bytes == 0) return DG_OK;
  if (hipHostMalloc(p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    *p = nullptr;
    return fail(DG_E_NOMEM, "hipHostMalloc of %llu bytes failed", (unsigned long long)bytes);
  }
  return DG_OK;
}

int dg_host_free(dg_engine* e, void* p) {
  if (!e) return fail(DG_E_INVAL, "null engine");
  if (!p) return DG_OK;
  TRY(set_device(e));
  HIP_TRY(hipStreamSynchronize(e->stream));  // no copy of this engine still reads or writes it
  HIP_TRY(hipHostFree(p));
  return DG_OK;
}

int dg_store_alloc(dg_engine* e, uint64_t cap, dg_store* s) {
  if (!e || !s) return fail(DG_E_INVAL, "dg_store_alloc: null argument");
  memset(s, 0, sizeof *s);
  const uint64_t c = cap ? cap : 1;
  void* p[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  const uint64_t w[5] = {8, 8, 8, 4, 8};
  for (int i = 0; i < 5; i++) {
    int rc = dg_buffer_alloc(e, c * w[i], &p[i]);
    if (rc != DG_OK) {
      for (int j = 0; j < i; j++) hipFree(p[j]);
      return rc;
    }
  }
  s->key = (uint64_t*)p[0];
  s->val = (uint64_t*)p[1];
  s->ts = (int64_t*)p[2];
  s->node = (uint32_t*)p[3];
  s->cnt = (uint64_t*)p[4];
  s->cap = cap;
  return DG_OK;
}

int dg_store_free(dg_engine* e, dg_store* s) {
  if (!e || !s) return fail(DG_E_INVAL, "dg_store_free: null argument");
  void* p[5] = {s->key, s->val, s->ts, s->node, s->cnt};
  for (int i = 0; i < 5; i++) TRY(dg_buffer_free(e, p[i]));
  memset(s, 0, sizeof *s);
  return DG_OK;
}

int dg_store_upload(dg_engine* e, const dg_store* host, dg_store* dev) {
  if (!e || !host || !dev) return fail(DG_E_INVAL, "dg_store_upload: null argument");
  if (dev->cap < host->n) return fail(DG_E_CAPACITY, "dg_store_upload: device cap too small");
  TRY(set_device(e));
  const uint64_t n = host->n;
  if (n) {
    HIP_TRY(hipMemcpyAsync(dev->key, host->key, n * 8, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(dev->val, host->val, n * 8, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(dev->ts, host->ts, n * 8, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(dev->node, host->node, n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(dev->cnt, host->cnt, n * 8, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  dev->n = n;
  return DG_OK;
}

int dg_store_download(dg_engine* e, const dg_store* dev, dg_store* host) {
  if (!e || !host || !dev) return fail(DG_E_INVAL, "dg_store_download: null argument");
  if (host->cap < dev->n) return fail(DG_E_CAPACITY, "dg_store_download: host cap too small");
  TRY(set_device(e));
  const uint64_t n = dev->n;
  if (n) {
    HIP_TRY(hipMemcpyAsync(host->key, dev->key, n * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(host->val, dev->val, n * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(host->ts, dev->ts, n * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(host->node, dev->node, n * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(host->cnt, dev->cnt, n * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  host->n = n;
  return DG_OK;
}

int dg_context_alloc(dg_engine* e, uint64_t cap, dg_context* c) {
  if (!e || !c) return fail(DG_E_INVAL, "dg_context_alloc: null argument");
  memset(c, 0, sizeof *c);
  void *pn = nullptr, *pc = nullptr;
  TRY(dg_buffer_alloc(e, (cap ? cap : 1) * 4, &pn));
  int rc = dg_buffer_alloc(e, (cap ? cap : 1) * 8, &pc);
  if (rc != DG_OK) {
    hipFree(pn);
    return rc;
  }
  c->node = (uint32_t*)pn;
  c->cnt = (uint64_t*)pc;
  c->cap = cap;
  return DG_OK;
}

int dg_context_free(dg_engine* e, dg_context* c) {
  if (!e || !c) return fail(DG_E_INVAL, "dg_context_free: null argument");
  TRY(dg_buffer_free(e, c->node));
  TRY(dg_buffer_free(e, c->cnt));
  memset(c, 0, sizeof *c);
  return DG_OK;
}

int dg_context_upload(dg_engine* e, const dg_context* host, dg_context* dev) {
  if (!e || !host || !dev) return fail(DG_E_INVAL, "dg_context_upload: null argument");
  if (dev->cap < host->n) return fail(DG_E_CAPACITY, "dg_context_upload: device cap too small");
  TRY(dg_copy_to_device(e, dev->node, host->node, host->n * 4));
  TRY(dg_copy_to_device(e, dev->cnt, host->cnt, host->n * 8));
  dev->n = host->n;
  dev->kind = host->kind;
  return DG_OK;
}

int dg_context_download(dg_engine* e, const dg_context* dev, dg_context* host) {
  if (!e || !host || !dev) return fail(DG_E_INVAL, "dg_context_download: null argument");
  if (host->cap < dev->n) return fail(DG_E_CAPACITY, "dg_context_download: host cap too small");
  TRY(dg_copy_to_host(e, host->node, dev->node, dev->n * 4));
  TRY(dg_copy_to_host(e, host->cnt, dev->cnt, dev->n * 8));
  host->n = dev->n;
  host->kind = dev->kind;
  return DG_OK;
}

}  // extern "C"
