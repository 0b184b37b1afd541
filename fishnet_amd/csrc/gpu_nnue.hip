// gpu_nnue.hip — C-ABI of libgpu_nnue.so (see include/gpu_nnue.h).
//
// Host side of the boundary that replaces the per-core Stockfish processes'
// static evaluation for batch workloads (/root/reference/src/stockfish.rs:36-47
// is the plugin API it sits beside).  Owns: the .nnue loader, device memory,
// one HIP stream per device, FEN packing, and the launch sequences of the
// kernels in kernels.hip.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "archive.h"
#include "host_board.h"
#include "kernels.h"
#include "sha256.h"

using namespace gn;

// ------------------------------------------------------------ errors ------
static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                               \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) return fail(GN_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                      __FILE__, __LINE__);                                          \
  } while (0)

namespace gn {
const Tables &host_tables() {
  static Tables T = [] {
    Tables t;
    init_tables(t);
    return t;
  }();
  return T;
}
} // namespace gn

// ----------------------------------------------------------- net file -----
struct HostNet {
  int L1 = 0;
  uint32_t hash = 0;
  std::vector<uint8_t> ft;    // [22528][ft_row_stride(L1)]
  std::vector<int16_t> bias;  // [L1], doubled
  std::vector<int8_t> w0, w1, w2;
  std::vector<int32_t> b0, b1, b2;
};

struct Reader {
  const uint8_t *p;
  size_t n, off = 0;
  bool take(void *dst, size_t k) {
    if (off + k > n) return false;
    memcpy(dst, p + off, k);
    off += k;
    return true;
  }
  bool u32(uint32_t &v) {
    uint8_t b[4];
    if (!take(b, 4)) return false;
    v = (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
    return true;
  }
  // signed LEB128 block ("COMPRESSED_LEB128", u32 byte count, payload)
  template <class Emit>
  bool leb(int bits, size_t count, Emit &&emit) {
    char magic[17];
    uint32_t nbytes;
    if (!take(magic, 17) || memcmp(magic, "COMPRESSED_LEB128", 17) || !u32(nbytes) || off + nbytes > n) return false;
    const uint8_t *q = p + off, *end = q + nbytes;
    for (size_t i = 0; i < count; ++i) {
      uint32_t r = 0;
      int shift = 0;
      for (;;) {
        if (q >= end || shift >= bits) return false;
        const uint8_t byte = *q++;
        r |= (uint32_t)(byte & 0x7f) << shift;
        shift += 7;
        if (!(byte & 0x80)) {
          if (shift < 32 && (byte & 0x40)) r |= ~((1u << shift) - 1u);
          break;
        }
      }
      emit(i, bits == 16 ? (int32_t)(int16_t)(uint16_t)r : (int32_t)r);
    }
    if (q != end) return false;
    off += nbytes;
    return true;
  }
};

static int parse_net(const uint8_t *data, size_t len, HostNet &h) {
  Reader r{data, len};
  uint32_t version, hash, dlen, fth;
  if (!r.u32(version) || version != NNUE_VERSION) return fail(GN_E_FORMAT, "not a Stockfish .nnue (version)");
  if (!r.u32(hash) || !r.u32(dlen) || r.off + dlen > len) return fail(GN_E_FORMAT, "bad .nnue header");
  r.off += dlen;
  if (!r.u32(fth)) return fail(GN_E_FORMAT, "truncated .nnue");
  int l1 = 0;
  for (int c = 32; c <= 4096 && !l1; c += 32)
    if (ft_hash(c) == fth && (ft_hash(c) ^ arch_hash(c)) == hash) l1 = c;
  if (!l1) return fail(GN_E_FORMAT, "network hash 0x%08x does not match a HalfKAv2_hm architecture", hash);
  if (l1 != 3072 && l1 != 1024 && l1 != 128) return fail(GN_E_FORMAT, "unsupported L1 width %d", l1);
  h.L1 = l1;
  h.hash = hash;
  const size_t RS = ft_row_stride((uint32_t)l1);
  h.ft.assign((size_t)FT_ROWS * RS, 0);
  h.bias.resize(l1);
  uint8_t *ft = h.ft.data();
  if (!r.leb(16, l1, [&](size_t i, int32_t v) { h.bias[i] = (int16_t)(uint16_t)(v * 2); }))
    return fail(GN_E_FORMAT, "bad feature-transformer biases");
  memcpy(ft + (size_t)FT_BIAS_ROW * RS, h.bias.data(), 2 * (size_t)l1);
  if (!r.leb(16, (size_t)l1 * FT_INPUTS, [&](size_t i, int32_t v) {
        const int16_t d = (int16_t)(uint16_t)(v * 2);
        memcpy(ft + (i / l1) * RS + 2 * (i % l1), &d, 2);
      }))
    return fail(GN_E_FORMAT, "bad feature-transformer weights");
  if (!r.leb(32, (size_t)PSQT_BUCKETS * FT_INPUTS, [&](size_t i, int32_t v) {
        memcpy(ft + (i / PSQT_BUCKETS) * RS + 2 * l1 + 4 * (i % PSQT_BUCKETS), &v, 4);
      }))
    return fail(GN_E_FORMAT, "bad PSQT weights");
  h.w0.resize((size_t)LAYER_STACKS * 16 * l1);
  h.w1.resize(LAYER_STACKS * 32 * 32);
  h.w2.resize(LAYER_STACKS * 32);
  h.b0.resize(LAYER_STACKS * 16);
  h.b1.resize(LAYER_STACKS * 32);
  h.b2.resize(LAYER_STACKS);
  const uint32_t ah = arch_hash(l1);
  for (int s = 0; s < LAYER_STACKS; ++s) {
    uint32_t hs;
    if (!r.u32(hs) || hs != ah) return fail(GN_E_FORMAT, "bad layer-stack hash in stack %d", s);
    bool ok = true;
    for (int i = 0; i < 16 && ok; ++i) ok = r.u32(reinterpret_cast<uint32_t &>(h.b0[s * 16 + i]));
    ok = ok && r.take(&h.w0[(size_t)s * 16 * l1], (size_t)16 * l1);
    for (int i = 0; i < 32 && ok; ++i) ok = r.u32(reinterpret_cast<uint32_t &>(h.b1[s * 32 + i]));
    ok = ok && r.take(&h.w1[s * 1024], 1024);
    ok = ok && r.u32(reinterpret_cast<uint32_t &>(h.b2[s]));
    ok = ok && r.take(&h.w2[s * 32], 32);
    if (!ok) return fail(GN_E_FORMAT, "truncated layer stack %d", s);
  }
  if (r.off != len) return fail(GN_E_FORMAT, "%zu trailing bytes after the network", len - r.off);
  return GN_OK;
}

// ----------------------------------------------------------- context ------
template <class T>
struct DevBuf {
  T *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    const size_t want = std::max(n, cap + cap / 2);
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    // (whole 16-B units: a kernel may read the aligned word holding a byte array's last byte,
    // plan_kernel's need / next-slot loads)
    hipError_t e = hipMalloc(&p, (std::max<size_t>(want, 1) * sizeof(T) + 15) & ~(size_t)15);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr, cap = 0;
  }
};

// The net outputs / selections of one evaluation (evaluate_on)
struct EvalBufs {
  DevBuf<int2> osm, obg;
  DevBuf<uint8_t> nsm, nbg;
  void release() { osm.release(), obg.release(), nsm.release(), nbg.release(); }
};

// ---- the drop-in's small batches ------------------------------------
// fishnet's GPU backend sends one game per gn_evaluate_batch (/root/reference/src/stockfish.rs:
// 36-47, src/main.rs:306-338: a chunk per worker call), ~80 positions, a few of them in check.
// The general path costs ~20 launches and three host round trips per call (the score rule's
// reply counts); on a one-device context a batch of <= 4,096 positions runs instead as one
// captured HIP graph per (size class, mode): upload from pinned memory, both levels of the
// in-check replies (reply_level_kernel: one workgroup selects from the boards, counts, scans and
// makes a level's replies; the levels are sized by their capacities, unused slots empty boards,
// so nothing waits for a count), one evaluation of the positions and both levels together, the
// two reductions (one workgroup), and the download of the overflow flag and the records.  One
// synchronisation per call.  A level with
// more replies than its capacity (nb / 2 + 256, nb / 4 + 256: beyond a game's) sets the flag and
// the call reruns on the general path.  Positions beyond n are empty boards (BAD_FEN records,
// never read back).
constexpr size_t FAST_NB0 = 128, FAST_MAX = 4096;
struct FastBatch {
  size_t nb = 0, c1 = 0, c2 = 0;
  int mode = -1;
  uint64_t gen = 0;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipEvent_t done = nullptr; // recorded behind each launch (the caller waits for it without d.mu)
  bool busy = false;         // a launch of this instance is in flight (d.mu)
  gn_board *h_in = nullptr; // pinned: nb boards
  gn_eval *h_out = nullptr; // pinned: one record holding the overflow flag, then nb records
  // the three levels one after another (in: nb boards, r1: c1 replies, r2: c2 replies of replies)
  // and their records behind the flag record, so that one evaluation covers them all
  DevBuf<gn_board> all;
  DevBuf<gn_eval> rec;
  gn_board *in = nullptr, *r1 = nullptr, *r2 = nullptr;
  gn_eval *out = nullptr, *e1 = nullptr, *e2 = nullptr;
  DevBuf<uint64_t> off0, off1;
  DevBuf<uint16_t> m1, m2;
  DevBuf<int32_t> sv1, sv2;
  EvalBufs eb;
  ~FastBatch() {
    if (done) (void)hipEventDestroy(done);
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    if (h_in) (void)hipHostFree(h_in);
    if (h_out) (void)hipHostFree(h_out);
    all.release(), rec.release();
    off0.release(), off1.release(), m1.release(), m2.release(), sv1.release(), sv2.release();
    eb.release();
  }
};

// The buffers one expansion's front half (child generation, classify, small net, plan) writes and
// its back half (row stream, finalize, score rule) reads: the expansion pipeline (expand_pipeline
// below) runs expansion k + 1's front on the device's second stream while expansion k's back
// runs, in the other set (swap_sets: the Dev's own fields are always the current set).
struct ExpSet {
  DevBuf<uint64_t> counts, offsets;
  DevBuf<uint32_t> owner;
  DevBuf<Board> unpacked;
  DevBuf<uint16_t> moves_tmp;
  const uint16_t *child_moves = nullptr;
  DevBuf<int2> pinfo, p_osm, p_obg;
  DevBuf<uint8_t> p_nsm, p_nbg;
  EvalBufs eb;
  DevBuf<gn_board> children;
  int chain_k = 1, slices = 1;
  bool planned = false;
  uint64_t etot = 0;
  void *scan_tmp = nullptr, *sort_tmp = nullptr; // (the two streams' scans / sorts run at once)
  size_t scan_bytes = 0, sort_bytes = 0;
  DevBuf<uint32_t> perr;            // the planned expansion's error word ...
  DevBuf<unsigned long long> pstat; // ... and pad count (each expansion of the pipeline its own)
  // the plan's output the row stream reads (GN_OPT_EXPAND_PIPELINE 2: the next plan runs beside
  // this expansion's row stream)
  DevBuf<uint64_t> ent, eoff;
  DevBuf<TileDesc> tiles;
  DevBuf<uint32_t> btiles, border;
  void release() {
    perr.release(), pstat.release();
    ent.release(), eoff.release(), tiles.release(), btiles.release(), border.release();
    counts.release(), offsets.release(), owner.release(), unpacked.release(), moves_tmp.release();
    pinfo.release(), p_osm.release(), p_obg.release(), p_nsm.release(), p_nbg.release(), eb.release();
    children.release();
    if (scan_tmp) (void)hipFree(scan_tmp);
    if (sort_tmp) (void)hipFree(sort_tmp);
    scan_tmp = sort_tmp = nullptr, scan_bytes = sort_bytes = 0;
  }
};

struct Dev {
  int id = 0;
  hipStream_t stream = nullptr;
  void *net_mem[2] = {nullptr, nullptr};
  NetDevice net[2] = {};
  bool has[2] = {false, false};
  Tables *tables = nullptr;
  EvalBufs eb; // evaluate_on's outputs
  DevBuf<int2> &osm = eb.osm, &obg = eb.obg;
  DevBuf<uint8_t> &nsm = eb.nsm, &nbg = eb.nbg;
  DevBuf<gn_board> io_boards, frontier[2];
  DevBuf<gn_eval> io_out, io_out2;
  DevBuf<uint64_t> counts, offsets;
  DevBuf<uint32_t> off32;
  DevBuf<uint16_t> moves, moves_tmp; // moves_tmp: when the caller keeps no moves
  DevBuf<uint32_t> owner;             // parent of each child (write_children scratch)
  DevBuf<Board> unpacked;             // the parents unpacked once (write_children scratch)
  const uint16_t *child_moves = nullptr; // the last generate_children's moves (finalize reads them)
  DevBuf<ChildDelta> deltas;
  DevBuf<uint64_t> kkeys, kkeys2; // king-sort keys
  DevBuf<uint32_t> kidx, kperm;   // king-sort permutation
  void *sort_tmp = nullptr;
  size_t sort_bytes = 0;
  DevBuf<int2> p_osm, p_obg;     // parent-side net outputs during expansion
  DevBuf<uint8_t> p_nsm, p_nbg;  // parent-side net selection during expansion
  DevBuf<unsigned long long> sum;
  DevBuf<uint8_t> nslot; // chained walk: child of parent i that is parent i + 1 (255: none)
  DevBuf<int32_t> part;  // column-sliced stream: fc_0 partial sums of the 3 slices (3 x positions x 16)
  DevBuf<int2> pinfo;    // ... and each position's (PSQT value, bucket) for the finish
  int chain_k = 1;          // block length of the current expansion (1: no chaining)
  int slices = 1;           // the current expansion's stream: column slices (3) or whole rows (1)
  bool part_locked = false; // a pipeline runs: part is in use by a back half (no reallocation)
  // planned expansion (stream.hip): per-parent entry bounds and their scan, the entry
  // lists, tile descriptors, the scratch-slot pool and the error word
  DevBuf<uint64_t> ebound, eoff;
  DevBuf<uint64_t> ent;           // the planned expansion's row entries (stream.hip)
  DevBuf<uint32_t> pool, perr;
  DevBuf<unsigned long long> pstat; // no-op entries the last planned expansion's plan inserted (GN_SCR_GAP)
  DevBuf<TileDesc> tiles;
  DevBuf<uint32_t> btiles; // tiles per block of the planned expansion
  DevBuf<uint16_t> bkeys, bkeys2; // block_order scratch
  DevBuf<uint32_t> bidx, border;  // block_order: identity, then the order
  uint64_t etot = 0;        // eoff[n] of the current expansion
  bool planned = false;     // the last expansion runs the planned kernels (perr is meaningful)
  void *scan_tmp = nullptr;
  size_t scan_bytes = 0;
  // Cross-stream ordering of the library-owned scratch above: every launch sequence
  // waits for the previous one when it runs on another stream (gn_*_device take a
  // caller stream and return while their kernels are still queued).
  hipEvent_t done = nullptr;
  hipStream_t done_on = nullptr;
  float plan_ms = 0, stream_ms = 0, finish_ms = 0; // the last timed planned expansion (GN_STAT_PLAN_NS /
                                                    // _STREAM_NS / _FINISH_NS)
  // the score rule's two levels of in-check replies (resolve_scores): selection, the selected
  // positions, their replies and the replies' records / rule values
  struct ScoreLevel {
    DevBuf<uint64_t> sel, pos, counts, offsets;
    DevBuf<uint32_t> idx, owner;
    DevBuf<gn_board> boards, children;
    DevBuf<uint16_t> moves;
    DevBuf<gn_eval> ce;
    DevBuf<int32_t> sv;
    void release() {
      sel.release(), pos.release(), counts.release(), offsets.release(), idx.release(), owner.release();
      boards.release(), children.release(), moves.release(), ce.release(), sv.release();
    }
  } lv[2];
  // the host-buffer calls' pipeline (expand_chunks): per chunk slot the parent / child
  // records and child moves a drain thread downloads on the copy stream while the next chunk
  // computes; the lichess replay's inputs and outputs (replay_games_kernel)
  hipStream_t copy = nullptr;
  hipEvent_t cev[2] = {nullptr, nullptr};
  DevBuf<gn_eval> po2[2], co2[2];
  DevBuf<gn_child> cc2[2]; // co2 packed as the host's 12-B child records (ABI v4)
  DevBuf<uint16_t> mv2[2];
  DevBuf<gn_board> roots, rboards, par;
  DevBuf<uint64_t> moff;
  DevBuf<uint16_t> codes, smoves;
  DevBuf<int32_t> rstatus;
  DevBuf<uint32_t> gidx;
  // stage times of the last host-buffer call on this device (GN_STAT_HOST_*), ms
  double t_upload = 0, t_replay = 0, t_compute = 0, t_download = 0, t_tail = 0;
  // the drop-in's small-batch graphs (FastBatch): two per size class (128 << k positions) and mode,
  // so that a second call's launch queues on the stream behind a first one in flight
  std::unique_ptr<FastBatch> fast[6][3][2];
  std::condition_variable fast_cv; // an instance's launch completed (its busy flag cleared; d.mu)
  // the expansion pipeline: the other buffer set, the front's stream and its two events (the
  // back's row stream done: the front may overwrite the plan's lists; the plan done)
  ExpSet alt;
  hipStream_t front = nullptr;
  hipEvent_t ev_streamed = nullptr, ev_planned = nullptr;
  std::mutex mu;
};

// The Dev's current expansion buffers <-> its other set (host-side pointers only: launches already
// queued keep the buffers they were given).
static void swap_sets(Dev &d) {
  ExpSet &x = d.alt;
  std::swap(d.counts, x.counts), std::swap(d.offsets, x.offsets), std::swap(d.owner, x.owner);
  std::swap(d.unpacked, x.unpacked), std::swap(d.moves_tmp, x.moves_tmp), std::swap(d.child_moves, x.child_moves);
  std::swap(d.pinfo, x.pinfo), std::swap(d.p_osm, x.p_osm), std::swap(d.p_obg, x.p_obg);
  std::swap(d.p_nsm, x.p_nsm), std::swap(d.p_nbg, x.p_nbg);
  std::swap(d.eb.osm, x.eb.osm), std::swap(d.eb.obg, x.eb.obg), std::swap(d.eb.nsm, x.eb.nsm), std::swap(d.eb.nbg, x.eb.nbg);
  std::swap(d.frontier[1], x.children);
  std::swap(d.chain_k, x.chain_k), std::swap(d.slices, x.slices), std::swap(d.planned, x.planned);
  std::swap(d.etot, x.etot);
  std::swap(d.scan_tmp, x.scan_tmp), std::swap(d.scan_bytes, x.scan_bytes);
  std::swap(d.sort_tmp, x.sort_tmp), std::swap(d.sort_bytes, x.sort_bytes);
  std::swap(d.perr, x.perr), std::swap(d.pstat, x.pstat);
  std::swap(d.ent, x.ent), std::swap(d.eoff, x.eoff), std::swap(d.tiles, x.tiles), std::swap(d.btiles, x.btiles);
  std::swap(d.border, x.border);
}

// Called under d.mu before a launch sequence on stream s / after it.
static hipError_t seq_begin(Dev &d, hipStream_t s) {
  if (d.done_on && d.done_on != s) return hipStreamWaitEvent(s, d.done, 0);
  return hipSuccess;
}
static hipError_t seq_end(Dev &d, hipStream_t s) {
  hipError_t e = hipEventRecord(d.done, s);
  if (e == hipSuccess) d.done_on = s;
  return e;
}
// After a synchronised planned expansion: its device error word (entry overflow or no
// scratch slot; neither can happen by construction, but a wrong result must not pass).
static int check_plan(Dev &d, hipStream_t s) {
  if (!d.planned || !d.perr.p) return GN_OK;
  uint32_t e = 0;
  HIP_TRY(hipMemcpyAsync(&e, d.perr.p, sizeof(e), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (e) return fail(GN_E_HIP, "planned expansion failed on the device (error bits 0x%x)", e);
  return GN_OK;
}

struct SeqGuard { // seq_begin now, seq_end when the scope ends (d.mu held throughout)
  Dev &d;
  hipStream_t s;
  hipError_t e;
  bool ended = false;
  SeqGuard(Dev &d_, hipStream_t s_) : d(d_), s(s_) { e = seq_begin(d, s); }
  // the sequence's end marker now, then wait for the stream: the call returns with its stream idle
  hipError_t finish() {
    ended = true;
    hipError_t r = seq_end(d, s);
    return r == hipSuccess ? hipStreamSynchronize(s) : r;
  }
  ~SeqGuard() {
    if (!ended) (void)seq_end(d, s);
  }
};

// Merged launches running at once (evaluate_coalesced).  Two (-DGN_MAX_LEADERS=2: a second
// leader's launch queues on the stream behind the first's, the small-batch graphs having two
// instances per class) measured the same 16-caller rate with 50 % more, smaller launches
// (round 6, profiles/r06/dropin_ab_r06w.txt): one at a time.
#ifndef GN_MAX_LEADERS
#define GN_MAX_LEADERS 1
#endif
constexpr int MAX_LEADERS = GN_MAX_LEADERS;
// One gn_evaluate_batch call waiting for, or in, a merged launch (evaluate_coalesced).
struct BatchReq {
  const gn_board *boards;
  size_t n;
  int mode;
  gn_eval *out;
  int rc = GN_OK;
  bool done = false;
  bool taken = false; // in a leader's launch (its thread waits for the result)
  char err[256] = ""; // (fixed size: copied while another caller's launch is marked busy, noexcept)
};

struct gn_ctx {
  std::vector<std::unique_ptr<Dev>> devs;
  // concurrent gn_evaluate_batch callers (fishnet's workers, one chunk per call) are merged
  // into one launch (evaluate_coalesced); GN_OPT_COALESCE
  struct {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<BatchReq *> q; // calls waiting for a launch
    int active = 0;            // launches running (<= MAX_LEADERS)
    uint64_t launches = 0, calls = 0;
  } co;
  bool coalesce = true;
  bool fast_batch = true;                  // GN_OPT_FAST_BATCH
  int pipeline = 2;                        // GN_OPT_EXPAND_PIPELINE (2: the next front beside the stream)
  std::atomic<uint64_t> graph_gen{0};      // bumped by every option / parameter change: the small-
                                           // batch graphs captured before it are rebuilt
  std::atomic<uint64_t> fast_runs{0}, fast_fallbacks{0};
  gn_eval_params P;
  bool incremental = true; // GN_OPT_INCREMENTAL_CHILDREN
  int swizzle = 9;          // GN_OPT_XCD_SWIZZLE bit mask: 1 small-net expansion, 2 batch evaluation,
                            // 4 / 8 big-net expansion (static eighths / XCD-local claiming)
  int king_sort = 1;        // GN_OPT_KING_SORT (1: batches of >= KING_SORT_MIN positions, 2: all)
  int chain = 81;           // GN_OPT_CHAIN (blocks of consecutive parents per workgroup)
  bool king_cache = true;   // GN_OPT_KING_CACHE
  int stream_slices = 3;    // GN_OPT_STREAM_SLICES (3 or 1)
  int64_t chunk_parents = 0; // GN_OPT_CHUNK_PARENTS (0: automatic)
  int l1[2] = {0, 0};
  uint32_t hash[2] = {0, 0};
  double t_parse = 0, t_total = 0; // the last host-buffer expansion call (GN_STAT_HOST_*), ms
};

enum { BIG = 0, SMALL = 1 };

static gn_eval_params default_params() {
  gn_eval_params P;
  P.small_net_threshold = 962;
  P.psqt_weight = 125;
  P.positional_weight = 131;
  P.reeval_threshold = 236;
  P.complexity_div_small = 18000;
  P.complexity_div_big = 18000;
  P.material_pawn_small = 535;
  P.material_pawn_big = 535;
  P.material_base = 77777;
  P.rule50_div = 212;
  P.value_clamp = 31506;
  const int32_t pv[5] = {208, 781, 825, 1276, 2538};
  memcpy(P.piece_value, pv, sizeof(pv));
  const double wa[4] = {-37.45051876, 121.19101539, -132.78783573, 420.70576692};
  memcpy(P.wdl_a, wa, sizeof(wa));
  P.wdl_material_min = 17;
  P.wdl_material_max = 78;
  P.wdl_material_anchor = 58;
  const int32_t ww[5] = {1, 3, 3, 5, 9};
  memcpy(P.wdl_piece_weight, ww, sizeof(ww));
  return P;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int upload_net(Dev &d, int which, const HostNet &h) {
  const size_t RS = ft_row_stride((uint32_t)h.L1);
  size_t off[10], o = 0;
  const int carry = h.L1 == 128 ? 0 : CARRY_SLOTS; // the chained walk's scratch rows
  // the PSQT weights once more as [bucket][row] (721 KB: L2-resident for the plan kernel's
  // scattered 4-byte reads, which would otherwise each touch a 6 KB FT row)
  std::vector<int32_t> psqt((size_t)PSQT_BUCKETS * FT_ROWS);
  for (size_t r = 0; r < (size_t)FT_ROWS; ++r)
    for (int b = 0; b < PSQT_BUCKETS; ++b)
      memcpy(&psqt[(size_t)b * FT_ROWS + r], h.ft.data() + r * RS + 2 * (size_t)h.L1 + 4 * b, 4);
  // fc_0 weights once more in the MFMA's operand order (stream.hip): per bucket and 64-wide
  // k-step, lane ln's 16 bytes (output ln & 15, inputs 16 (ln >> 4) .. + 15) at 16 ln, so a
  // wave's k-step is one contiguous 1 KiB (8 whole lines) instead of 16 pieces of 64 B
  const int KS = h.L1 / 64;
  std::vector<int8_t> w0f(h.w0.size());
  for (int b = 0; b < LAYER_STACKS; ++b)
    for (int ks = 0; ks < KS; ++ks)
      for (int ln = 0; ln < 64; ++ln)
        memcpy(&w0f[(((size_t)b * KS + ks) * 64 + ln) * 16],
               &h.w0[((size_t)b * 16 + (ln & 15)) * h.L1 + 64 * (size_t)ks + 16 * (ln >> 4)], 16);
  const size_t sz[10] = {((size_t)FT_ROWS + 4 * (size_t)carry + 128 * (size_t)carry + (carry ? 1 : 0)) * RS, h.bias.size() * 2, h.w0.size(), h.b0.size() * 4,
                         h.w1.size(), h.b1.size() * 4, h.w2.size(), h.b2.size() * 4, psqt.size() * 4, w0f.size()};
  const void *src[10] = {h.ft.data(), h.bias.data(), h.w0.data(), h.b0.data(),
                         h.w1.data(), h.b1.data(), h.w2.data(), h.b2.data(), psqt.data(), w0f.data()};
  for (int i = 0; i < 10; ++i) off[i] = o, o += align256(sz[i]);
  uint8_t *m = nullptr;
  if (hipMalloc(&m, o) != hipSuccess) return fail(GN_E_NOMEM, "device allocation of %zu bytes failed", o);
  d.net_mem[which] = m;
  for (int i = 0; i < 10; ++i)
    HIP_TRY(hipMemcpy(m + off[i], src[i], i == 0 ? (size_t)FT_ROWS * RS : sz[i], hipMemcpyHostToDevice));
  if (carry) HIP_TRY(hipMemset(m + off[0] + (size_t)FT_ROWS * RS, 0, 4 * (size_t)carry * RS));
  if (carry) HIP_TRY(hipMemset(m + off[0] + (size_t)ZERO_ROW * RS, 0, RS)); // the zero row
  NetDevice &n = d.net[which];
  n.L1 = h.L1;
  n.row_stride = (uint32_t)RS;
  n.carry_slots = carry;
  n.kc_slots = carry;
  n.ft = m + off[0];
  n.bias = reinterpret_cast<const int16_t *>(m + off[1]);
  n.w0 = reinterpret_cast<const int8_t *>(m + off[2]);
  n.b0 = reinterpret_cast<const int32_t *>(m + off[3]);
  n.w1 = reinterpret_cast<const int8_t *>(m + off[4]);
  n.b1 = reinterpret_cast<const int32_t *>(m + off[5]);
  n.w2 = reinterpret_cast<const int8_t *>(m + off[6]);
  n.b2 = reinterpret_cast<const int32_t *>(m + off[7]);
  n.psqt = reinterpret_cast<const int32_t *>(m + off[8]);
  n.w0f = reinterpret_cast<const int8_t *>(m + off[9]);
  d.has[which] = true;
  return GN_OK;
}

static void destroy(gn_ctx *ctx) {
  if (!ctx) return;
  for (auto &dp : ctx->devs) {
    Dev &d = *dp;
    (void)hipSetDevice(d.id);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    for (void *m : d.net_mem)
      if (m) (void)hipFree(m);
    if (d.tables) (void)hipFree(d.tables);
    d.osm.release(), d.obg.release(), d.nsm.release(), d.nbg.release();
    d.io_boards.release(), d.frontier[0].release(), d.frontier[1].release();
    d.io_out.release(), d.io_out2.release(), d.counts.release(), d.offsets.release();
    d.off32.release(), d.moves.release(), d.sum.release(), d.deltas.release();
    d.moves_tmp.release(), d.owner.release(), d.unpacked.release();
    d.p_osm.release(), d.p_obg.release(), d.p_nsm.release(), d.p_nbg.release();
    d.part.release(), d.pinfo.release(), d.alt.release();
    if (d.front) (void)hipStreamSynchronize(d.front), (void)hipStreamDestroy(d.front);
    if (d.ev_streamed) (void)hipEventDestroy(d.ev_streamed);
    if (d.ev_planned) (void)hipEventDestroy(d.ev_planned);
    if (d.scan_tmp) (void)hipFree(d.scan_tmp);
    if (d.sort_tmp) (void)hipFree(d.sort_tmp);
    d.kkeys.release(), d.kkeys2.release(), d.kidx.release(), d.kperm.release();
    d.nslot.release();
    d.ebound.release(), d.eoff.release(), d.ent.release(), d.pool.release(), d.perr.release(), d.tiles.release(), d.btiles.release();
    d.pstat.release();
    d.bkeys.release(), d.bkeys2.release(), d.bidx.release(), d.border.release();
    d.lv[0].release(), d.lv[1].release();
    for (auto &row : d.fast)
      for (auto &pair : row)
        for (auto &f : pair) f.reset();
    for (int i = 0; i < 2; ++i) {
      d.po2[i].release(), d.co2[i].release(), d.cc2[i].release(), d.mv2[i].release();
      if (d.cev[i]) (void)hipEventDestroy(d.cev[i]);
    }
    d.roots.release(), d.rboards.release(), d.par.release(), d.moff.release(), d.codes.release();
    d.smoves.release(), d.rstatus.release(), d.gidx.release();
    if (d.copy) (void)hipStreamSynchronize(d.copy), (void)hipStreamDestroy(d.copy);
    if (d.done) (void)hipEventDestroy(d.done);
    if (d.stream) (void)hipStreamDestroy(d.stream);
  }
  delete ctx;
}

static int create(const uint8_t *big, size_t big_len, const uint8_t *small, size_t small_len, const int *devices,
                  int n_devices, gn_ctx **out) {
  if (!out) return fail(GN_E_INVALID, "out is NULL");
  *out = nullptr;
  if (!big && !small) return fail(GN_E_INVALID, "no network given");
  HostNet hn[2];
  if (big) {
    int rc = parse_net(big, big_len, hn[BIG]);
    if (rc) return rc;
  }
  if (small) {
    int rc = parse_net(small, small_len, hn[SMALL]);
    if (rc) return rc;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(GN_E_NODEVICE, "no HIP device visible");
  std::vector<int> ids;
  if (devices && n_devices > 0) ids.assign(devices, devices + n_devices);
  else ids.push_back(0);
  std::unique_ptr<gn_ctx, void (*)(gn_ctx *)> ctx(new gn_ctx(), destroy);
  ctx->P = default_params();
  for (int w = 0; w < 2; ++w) ctx->l1[w] = hn[w].L1, ctx->hash[w] = hn[w].hash;
  for (int id : ids) {
    if (id < 0 || id >= count) return fail(GN_E_NODEVICE, "device %d out of range (%d visible)", id, count);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, id));
    if (!strstr(prop.gcnArchName, "gfx950"))
      return fail(GN_E_NODEVICE, "device %d is %s; libgpu_nnue is built for gfx950 only", id, prop.gcnArchName);
    ctx->devs.emplace_back(new Dev());
    Dev &d = *ctx->devs.back();
    d.id = id;
    HIP_TRY(hipSetDevice(id));
    HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&d.done, hipEventDisableTiming));
    HIP_TRY(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
#ifdef GN_AB_FRONT_PRIORITY // A/B: the pipeline's front stream at the device's highest priority
    {
      int least = 0, greatest = 0;
      HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIP_TRY(hipStreamCreateWithPriority(&d.front, hipStreamNonBlocking, greatest));
    }
#else
    HIP_TRY(hipStreamCreateWithFlags(&d.front, hipStreamNonBlocking));
#endif
    HIP_TRY(hipEventCreateWithFlags(&d.ev_streamed, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_planned, hipEventDisableTiming));
    for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreateWithFlags(&d.cev[i], hipEventDisableTiming));
#ifdef GN_AB_AUX_STREAMS // A/B only: two extra streams, as the removed range pipeline had
    {
      hipStream_t x[2];
      for (int i = 0; i < 2; ++i) HIP_TRY(hipStreamCreateWithFlags(&x[i], hipStreamNonBlocking));
    }
#endif
    HIP_TRY(hipMalloc(&d.tables, sizeof(Tables)));
    HIP_TRY(d.perr.ensure(1)); // the planned expansion's error word and pad count (both sets)
    HIP_TRY(d.pstat.ensure(1));
    HIP_TRY(d.alt.perr.ensure(1));
    HIP_TRY(d.alt.pstat.ensure(1));
    HIP_TRY(hipMemset(d.alt.perr.p, 0, sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(d.tables, &host_tables(), sizeof(Tables), hipMemcpyHostToDevice));
    for (int w = 0; w < 2; ++w)
      if (hn[w].L1) {
        int rc = upload_net(d, w, hn[w]);
        if (rc) return rc;
      }
  }
  *out = ctx.release();
  return GN_OK;
}

static bool read_file(const char *path, std::vector<uint8_t> &buf) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  buf.resize(n > 0 ? (size_t)n : 0);
  bool ok = n >= 0 && fread(buf.data(), 1, buf.size(), f) == buf.size();
  fclose(f);
  return ok;
}

// ---------------------------------------------------------- launches ------
struct KernelTimes {
  hipEvent_t ev[10];
  bool on = false;
};

// Launch sequence of one evaluation.  ev (optional) = 5 events recorded between
// the stages [classify(+)] [small net (+reeval)] [big net] [finalize].
// score: the records are positions (the score rule's static part; resolve_scores does the
// in-check ones) rather than child records; counts (optional): their legal-move counts.
// eb (optional): the net outputs and selections in these buffers instead of the device's (the
// drop-in's captured small-batch graphs own theirs, FastBatch); sort false: no king sort.
static int evaluate_on(gn_ctx *ctx, Dev &d, const gn_board *b, size_t n, int mode, gn_eval *out, hipStream_t s,
                       hipEvent_t *ev, unsigned long long *rows_out = nullptr, int score = 1,
                       const uint64_t *counts = nullptr, EvalBufs *eb = nullptr, bool sort = true) {
  if (mode < GN_MODE_FULL || mode > GN_MODE_SMALL) return fail(GN_E_INVALID, "bad mode %d", mode);
  if ((mode != GN_MODE_SMALL && !d.has[BIG]) || (mode != GN_MODE_BIG && !d.has[SMALL]))
    return fail(GN_E_NONET, "mode %d needs a network that is not loaded", mode);
  if (!n) return GN_OK;
  EvalBufs &B = eb ? *eb : d.eb;
  DevBuf<int2> &osm = B.osm, &obg = B.obg;
  DevBuf<uint8_t> &nsm = B.nsm, &nbg = B.nbg;
  if (mode != GN_MODE_BIG) HIP_TRY(osm.ensure(n));
  if (mode != GN_MODE_SMALL) HIP_TRY(obg.ensure(n));
  if (mode == GN_MODE_FULL) {
    HIP_TRY(nsm.ensure(n));
    HIP_TRY(nbg.ensure(n));
  }
  auto mark = [&](int k) -> hipError_t { return ev ? hipEventRecord(ev[k], s) : hipSuccess; };
  const gn_eval_params &P = ctx->P;
  HIP_TRY(mark(0)); // (mode FULL's selection runs inside the small net's launch: launch_eval_net cls)
  const uint32_t *perm = nullptr;
  // a small batch (one game, a handful of in-check replies) gains nothing from the order and
  // would pay the sort's launches on its latency (bench.py secondary.dropin)
  constexpr size_t KING_SORT_MIN = 1024;
  if (sort && (ctx->king_sort == 2 || (ctx->king_sort == 1 && n >= KING_SORT_MIN))) {
    if (n > 0x7FFFFFFFull) return fail(GN_E_INVALID, "king sort supports < 2^31 positions per call");
    HIP_TRY(d.kkeys.ensure(n));
    HIP_TRY(d.kkeys2.ensure(n));
    HIP_TRY(d.kidx.ensure(n));
    HIP_TRY(d.kperm.ensure(n));
    HIP_TRY(king_sort(b, n, d.kkeys.p, d.kidx.p, d.kkeys2.p, d.kperm.p, mode != GN_MODE_SMALL, d.sort_tmp,
                      d.sort_bytes, s));
    perm = d.kperm.p;
  }
  const int swz = (ctx->swizzle >> 1) & 1;
  HIP_TRY(mark(1));
  if (mode != GN_MODE_BIG)
    HIP_TRY(launch_eval_net(d.net[SMALL], b, nullptr, n, osm.p, perm, swz, s, mode == GN_MODE_SMALL ? rows_out : nullptr,
                            mode == GN_MODE_FULL ? &P : nullptr, nsm.p, nbg.p));
  HIP_TRY(mark(2));
  if (mode != GN_MODE_SMALL)
    HIP_TRY(launch_eval_net(d.net[BIG], b, mode == GN_MODE_FULL ? nbg.p : nullptr, n, obg.p, perm, swz, s,
                            rows_out));
  HIP_TRY(mark(3));
  HIP_TRY(launch_finalize(b, n, mode, osm.p, obg.p, nsm.p, nbg.p, P, d.tables, out, s, score, counts));
  HIP_TRY(mark(4));
  return GN_OK;
}

static Dev *slot(gn_ctx *ctx, int s) {
  if (!ctx || s < 0 || s >= (int)ctx->devs.size()) return nullptr;
  return ctx->devs[s].get();
}

template <class F>
static void parallel_for(size_t n, size_t grain, F &&f) {
  unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  size_t chunks = std::min<size_t>(hw, (n + grain - 1) / std::max<size_t>(grain, 1));
  if (chunks <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  size_t per = (n + chunks - 1) / chunks;
  for (size_t c = 0; c < chunks; ++c) {
    size_t lo = c * per, hi = std::min(n, lo + per);
    if (lo < hi) th.emplace_back([=, &f] { f(lo, hi); });
  }
  for (auto &t : th) t.join();
}

// Child generation: counts -> exclusive scan (d.offsets, n + 1) -> children
// boards (+ moves, + ChildDelta when deltas is non-null).  *total = children.
// ev (optional) gets 3 events: after count+scan, after the host read of the
// total, after write_children.
// Block length of the chained walk for an n-parent expansion: GN_OPT_CHAIN, shortened
// (to >= 2) when the blocks would not fill the resident workgroups; 1 = off.
static int chain_len(const gn_ctx *ctx, Dev &d, size_t n) {
  if (!ctx->incremental || (ctx->chain >= -1 && ctx->chain <= 1) || !d.has[BIG] || !d.net[BIG].carry_slots)
    return 1;
  if (ctx->chain < 0) return -ctx->chain; // exact (tests)
  // keep >= 2048 blocks (8 per resident workgroup) when the batch allows
  size_t k = (size_t)ctx->chain;
  if ((n + k - 1) / k < 2048) k = std::max<size_t>(2, std::min(k, n / 2048));
  return (int)k;
}

// The big net's expansion (modes FULL / BIG) runs planned (stream.hip).
// (Round 2's pipeline of block ranges on two streams, range c + 1's child generation and plan
// under range c's row stream, took the same time as the serial order, 296 vs 259 + 19 + 15.5
// + 5 ms: the overlapped kernels slow the row stream by what they add; it was removed.)
static bool plan_path(const gn_ctx *ctx, const Dev &d, int mode) {
  return mode != GN_MODE_SMALL && ctx->incremental && d.has[BIG] &&
         (d.net[BIG].L1 == 3072 || d.net[BIG].L1 == 1024);
}

// finalize of the n parents and total children (their net outputs in the Dev buffers)
// (score_parents: the parents are positions with the score rule; the children are child records)
// (sliced: the big net's outputs are the sliced stream's partial sums, positions = parents then
// children, which finalize finishes itself)
static int finalize_all(gn_ctx *ctx, Dev &d, const gn_board *parents, const gn_board *children, int mode,
                        gn_eval *parent_out, gn_eval *child_out, size_t n, size_t total, hipStream_t s,
                        bool score_parents, bool sliced = false) {
  const gn_eval_params &P = ctx->P;
  const SlicedOut sc = {&d.net[BIG], d.part.p, d.pinfo.p, (uint64_t)(n + total), (uint64_t)n},
                  sp = {&d.net[BIG], d.part.p, d.pinfo.p, (uint64_t)(n + total), 0};
  // children from their parents as write_children unpacked them
  const bool fast = d.child_moves != nullptr;
  HIP_TRY(launch_finalize(children, total, mode, d.osm.p, d.obg.p, d.nsm.p, d.nbg.p, P, d.tables, child_out, s, 0,
                          nullptr, fast ? d.owner.p : nullptr, fast ? d.child_moves : nullptr,
                          fast ? d.unpacked.p : nullptr, sliced ? &sc : nullptr));
  if (parent_out) // the parents' legal-move counts are generate_children's
    HIP_TRY(launch_finalize(parents, n, mode, d.p_osm.p, d.p_obg.p, d.p_nsm.p, d.p_nbg.p, P, d.tables, parent_out, s,
                            score_parents ? 1 : 0, d.counts.p, nullptr, nullptr, nullptr, sliced ? &sp : nullptr));
  return GN_OK;
}

// Legal-child count of n boards (a capacity query), synchronously.
static hipError_t count_children(Dev &d, const gn_board *parents, size_t n, hipStream_t s, size_t *total) {
  hipError_t e;
  if ((e = d.counts.ensure(n + 1)) != hipSuccess || (e = d.offsets.ensure(n + 1)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(d.counts.p + n, 0, sizeof(uint64_t), s)) != hipSuccess) return e;
  if ((e = launch_count_children(parents, n, d.tables, d.counts.p, s)) != hipSuccess) return e;
  if ((e = exclusive_scan_u64(d.counts.p, d.offsets.p, n + 1, d.scan_tmp, d.scan_bytes, s)) != hipSuccess) return e;
  uint64_t t = 0;
  if ((e = hipMemcpyAsync(&t, d.offsets.p + n, sizeof(t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  *total = (size_t)t;
  return hipSuccess;
}

// skip_internal: the planned big-net path reads no child board after this (finalize makes each
// child from its unpacked parent and move), so library-internal child boards are not written.
static int generate_children(Dev &d, const gn_board *parents, size_t n, gn_board *children_or_null, size_t cap,
                             uint16_t *moves, bool want_deltas, size_t *total, hipStream_t s, hipEvent_t *ev,
                             unsigned long long *rows = nullptr, int chain_k = 1, bool plan = false,
                             bool skip_internal = false) {
  d.chain_k = want_deltas ? chain_k : 1;
  d.planned = want_deltas && plan;
  if (d.planned) { // a stale error bit of an earlier expansion must not fail this one
    HIP_TRY(hipMemsetAsync(d.perr.p, 0, sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(d.pstat.p, 0, sizeof(unsigned long long), s));
  }
  if (d.chain_k > 1) HIP_TRY(d.nslot.ensure(n));
  HIP_TRY(d.counts.ensure(n + 1));
  HIP_TRY(d.offsets.ensure(n + 1));
  HIP_TRY(hipMemsetAsync(d.counts.p + n, 0, sizeof(uint64_t), s));
  if (d.planned) {
    HIP_TRY(d.ebound.ensure(n + 1));
    HIP_TRY(d.eoff.ensure(n + 1));
    HIP_TRY(hipMemsetAsync(d.ebound.p + n, 0, sizeof(uint64_t), s));
  }
  HIP_TRY(launch_count_children(parents, n, d.tables, d.counts.p, s, d.planned ? d.ebound.p : nullptr));
  HIP_TRY(exclusive_scan_u64(d.counts.p, d.offsets.p, n + 1, d.scan_tmp, d.scan_bytes, s));
  if (d.planned) HIP_TRY(exclusive_scan_u64(d.ebound.p, d.eoff.p, n + 1, d.scan_tmp, d.scan_bytes, s));
  if (ev) HIP_TRY(hipEventRecord(ev[0], s));
  uint64_t t = 0;
  HIP_TRY(hipMemcpyAsync(&t, d.offsets.p + n, sizeof(t), hipMemcpyDeviceToHost, s));
  if (d.planned) HIP_TRY(hipMemcpyAsync(&d.etot, d.eoff.p + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *total = (size_t)t;
  if (ev) HIP_TRY(hipEventRecord(ev[1], s));
  if ((children_or_null || moves) && t > cap) // caller-owned child buffers hold cap entries
    return fail(GN_E_CAPACITY, "%zu children exceed capacity %zu", (size_t)t, cap);
  gn_board *children = children_or_null;
  const bool skip_boards = !children_or_null && d.planned && skip_internal;
  if (!children && !skip_boards) {
    HIP_TRY(d.frontier[1].ensure(std::max<size_t>(t, 1)));
    children = d.frontier[1].p;
  }
  if (want_deltas) HIP_TRY(d.deltas.ensure(std::max<size_t>(t, 1)));
  HIP_TRY(d.owner.ensure(std::max<size_t>(t, 1)));
  HIP_TRY(d.unpacked.ensure(std::max<size_t>(n, 1)));
  if (!moves) {
    HIP_TRY(d.moves_tmp.ensure(std::max<size_t>(t, 1)));
    moves = d.moves_tmp.p;
  }
  d.child_moves = moves;
  if (t) {
    HIP_TRY(launch_write_children(parents, n, d.tables, d.offsets.p, 0, t, children, moves, d.owner.p,
                                  want_deltas ? d.deltas.p : nullptr, d.chain_k > 1 ? d.nslot.p : nullptr, d.chain_k,
                                  rows, s, d.unpacked.p));
  }
  if (ev) HIP_TRY(hipEventRecord(ev[2], s));
  return GN_OK;
}

// Evaluate parents + children after generate_children.  Incremental: the
// expand_eval kernels (one workgroup per parent, children from the parent
// accumulators); otherwise every child is a full refresh (evaluate_on).
// ev (optional) gets 5 events: after classify, after the small net (+reeval),
// after the big net, after finalize, and (planned path) between its plan and stream kernels.
// score_parents: the parents are positions (the score rule's static part; callers run
// resolve_scores on them) rather than child records (depth 2's level 2).
// phases: EXP_FRONT (classify, the small net, the big net's plan) and / or EXP_BACK (the big net's
// row stream, finalize); the expansion pipeline runs the two on different streams.  ev (optional):
// [0] after classify, [1] after the small net, [2] after the big net, [3] after finalize, [4] the
// plan -> stream boundary, [6] after the stream launches, [7] (EXP_BACK alone) the stream's start.
// streamed (without ev): recorded after the stream launches (the pipeline's next front waits for it).
constexpr int EXP_FRONT = 1, EXP_BACK = 2;
static int expand_evaluate(gn_ctx *ctx, Dev &d, const gn_board *parents, size_t n, const gn_board *children,
                           size_t total, int mode, gn_eval *parent_out, gn_eval *child_out, hipStream_t s,
                           hipEvent_t *ev, unsigned long long *rows_out = nullptr, bool score_parents = true,
                           int phases = EXP_FRONT | EXP_BACK, hipEvent_t streamed = nullptr) {
  if (mode < GN_MODE_FULL || mode > GN_MODE_SMALL) return fail(GN_E_INVALID, "bad mode %d", mode);
  if ((mode != GN_MODE_SMALL && !d.has[BIG]) || (mode != GN_MODE_BIG && !d.has[SMALL]))
    return fail(GN_E_NONET, "mode %d needs a network that is not loaded", mode);
  if (!ctx->incremental) {
    if (!(phases & EXP_BACK)) return GN_OK; // (no front half: every child is a full refresh)
    if (total) {
      int rc = evaluate_on(ctx, d, children, total, mode, child_out, s, nullptr, nullptr, 0);
      if (rc) return rc;
    }
    return parent_out ? evaluate_on(ctx, d, parents, n, mode, parent_out, s, nullptr, nullptr, score_parents ? 1 : 0,
                                    d.counts.p)
                      : GN_OK;
  }
  auto mark = [&](int k) -> hipError_t { return ev ? hipEventRecord(ev[k], s) : hipSuccess; };
  const gn_eval_params &P = ctx->P;
  const uint64_t *off = d.offsets.p;
  const ChildDelta *dl = d.deltas.p;
  const bool f = mode == GN_MODE_FULL;
  const size_t K = (size_t)std::max(1, d.chain_k), nblk = (n + K - 1) / K;
  // ---- the front half: selections, the small net, the plan (the stream's lists and tiles)
  if (phases & EXP_FRONT) {
    const size_t nt = std::max<size_t>(total, 1);
    if (mode != GN_MODE_BIG) {
      HIP_TRY(d.osm.ensure(nt));
      HIP_TRY(d.p_osm.ensure(n));
    }
    if (mode != GN_MODE_SMALL) {
      HIP_TRY(d.obg.ensure(nt));
      HIP_TRY(d.p_obg.ensure(n));
    }
    if (f) {
      HIP_TRY(d.nsm.ensure(nt));
      HIP_TRY(d.nbg.ensure(nt));
      HIP_TRY(d.p_nsm.ensure(n));
      HIP_TRY(d.p_nbg.ensure(n));
      HIP_TRY(launch_classify(parents, n, P, d.p_nsm.p, d.p_nbg.p, s));
      HIP_TRY(launch_classify(children, total, P, d.nsm.p, d.nbg.p, s));
    }
    HIP_TRY(mark(0));
    if (mode != GN_MODE_BIG) {
      HIP_TRY(launch_expand_net(d.net[SMALL], parents, n, off, children, dl, f ? d.p_nsm.p : nullptr,
                                f ? d.nsm.p : nullptr, d.p_osm.p, d.osm.p, ctx->swizzle & 1, s));
      if (f) {
        HIP_TRY(launch_reeval(d.p_osm.p, d.p_nsm.p, n, P, d.p_nbg.p, s));
        HIP_TRY(launch_reeval(d.osm.p, d.nsm.p, total, P, d.nbg.p, s));
      }
    }
    HIP_TRY(mark(1));
    d.slices = 1;
    if (mode != GN_MODE_SMALL && d.planned) {
      HIP_TRY(d.ent.ensure(d.etot + (size_t)ENT_SPARE * (nblk + 1)));
      HIP_TRY(d.tiles.ensure((n + total) / 16 + (K + 2) * nblk + 2));
      HIP_TRY(d.btiles.ensure(nblk + 1));
      HIP_TRY(d.pool.ensure(88)); // 8 XCDs x 8 words of scratch-slot bits, then 8 block claim counters
      int slices = d.net[BIG].L1 == 3072 && ctx->stream_slices == 3 ? 3 : 1;
      // the sliced stream's partial sums cost 200 B per position (include/gpu_nnue.h,
      // GN_OPT_STREAM_SLICES); when they do not fit, the whole-row stream gives the same results
      // (part_locked: a pipelined front, beside the back half of the previous expansion that reads
      // part -- it may not reallocate it; when it is too small this expansion streams whole rows)
      if (slices > 1) {
        const size_t need = (size_t)GN_PART_SLICES * 16 * (n + total);
        bool ok = d.part_locked ? d.part.cap >= need : d.part.ensure(need) == hipSuccess;
        ok = ok && d.pinfo.ensure(n + total) == hipSuccess;
        if (!ok) {
          (void)hipGetLastError(); // (the failed allocation's error is not the call's)
          if (!d.part_locked) d.part.release();
          d.pinfo.release();
          slices = 1;
        }
      }
      d.slices = slices;
      // XCD-local block order
      if (ctx->king_sort && nblk > 1) {
        HIP_TRY(d.bkeys.ensure(nblk));
        HIP_TRY(d.bkeys2.ensure(nblk));
        HIP_TRY(d.bidx.ensure(nblk));
        HIP_TRY(d.border.ensure(nblk));
        HIP_TRY(block_order(parents, n, (uint32_t)K, (uint32_t)nblk, d.bkeys.p, d.bidx.p, d.bkeys2.p, d.border.p,
                            d.sort_tmp, d.sort_bytes, s));
      }
      HIP_TRY(launch_plan_stream(d.net[BIG], parents, n, off, dl, f ? d.p_nbg.p : nullptr, f ? d.nbg.p : nullptr,
                                 d.p_obg.p, d.obg.p, 0, d.chain_k > 1 ? d.nslot.p : nullptr, d.chain_k,
                                 ctx->king_cache ? 1 : 0, d.eoff.p, d.ent.p, d.tiles.p, d.btiles.p, d.pool.p, d.perr.p,
                                 rows_out, d.pstat.p, 0, nblk, nullptr, ev ? ev[4] : nullptr, s, slices,
                                 slices > 1 ? d.part.p : nullptr, n + total, slices > 1 ? d.pinfo.p : nullptr,
                                 nullptr, false, PLAN_PHASE));
    }
  }
  if (!(phases & EXP_BACK)) return GN_OK;
  // ---- the back half: the big net's row stream, finalize
  bool fused = false; // the sliced stream's finish runs inside finalize
  if (mode != GN_MODE_SMALL) {
    if (d.planned) {
      const int slices = d.slices;
      const uint32_t *order = ctx->king_sort && nblk > 1 ? d.border.p : nullptr;
      HIP_TRY(hipMemsetAsync(d.pool.p, 0, 88 * sizeof(uint32_t), s)); // per stream launch (<= 3)
#ifndef GN_AB_FINISH_SEPARATE // A/B (round 4): slice_finish_kernel, then finalize
      fused = slices > 1;
#endif
      if (ev && (phases & EXP_FRONT) == 0) HIP_TRY(hipEventRecord(ev[7], s)); // (the pipeline: the stream's start)
      HIP_TRY(launch_plan_stream(d.net[BIG], parents, n, off, dl, f ? d.p_nbg.p : nullptr, f ? d.nbg.p : nullptr,
                                 d.p_obg.p, d.obg.p, (ctx->swizzle >> 2) & 1 ? 1 : (ctx->swizzle >> 3) & 1 ? 2 : 0,
                                 d.chain_k > 1 ? d.nslot.p : nullptr, d.chain_k,
                                 ctx->king_cache ? 1 : 0, d.eoff.p, d.ent.p, d.tiles.p, d.btiles.p, d.pool.p, d.perr.p,
                                 rows_out, d.pstat.p, 0, nblk, order, nullptr, s, slices,
                                 slices > 1 ? d.part.p : nullptr, n + total, slices > 1 ? d.pinfo.p : nullptr,
                                 ev ? ev[6] : streamed, !fused, STREAM_PHASE));
    } else { // a 128-wide net loaded as the big net
      HIP_TRY(launch_expand_net(d.net[BIG], parents, n, off, children, dl, f ? d.p_nbg.p : nullptr,
                                f ? d.nbg.p : nullptr, d.p_obg.p, d.obg.p, ctx->swizzle & 1, s));
    }
  }
  HIP_TRY(mark(2));
  int rc = finalize_all(ctx, d, parents, children, mode, parent_out, child_out, n, total, s, score_parents, fused);
  if (rc) return rc;
  HIP_TRY(mark(3));
  return GN_OK;
}

// ---------------------------------------------------------- score rule ---
// The in-check part of the score rule (include/gpu_nnue.h, gn_eval.score): for every scored
// position of out[0, n) in check with a legal move (finalize set the rest), its legal
// replies are generated and evaluated as positions on the device, the replies in check
// are resolved one level down (depth 2 -> 1; at depth 0 a reply keeps its static value),
// and score_reduce_kernel takes the negamax over them.  sv_out (optional): the positions'
// rule values for the level above.  Synchronous (the selection's and the replies' counts
// size the next launches); a batch without such positions costs one select + scan.
// Stockfish has no static evaluation in check (Eval::evaluate asserts !checkers) and
// always prints a score from its search; fishnet requires one for every analysed
// position (/root/reference/src/stockfish.rs:366-368, src/ipc.rs:56).
// replies (optional, an expansion's parents): every position's legal replies are already
// evaluated (child records / moves at d.offsets, the parents unpacked in d.unpacked); they are
// reused instead of generated and evaluated again.
struct Replies {
  const gn_eval *rec;
  const uint16_t *moves;
};
static int resolve_scores(gn_ctx *ctx, Dev &d, const gn_board *boards, size_t n, int mode, gn_eval *out,
                          int32_t *sv_out, hipStream_t s, int depth = 2, const Replies *replies = nullptr) {
  if (!n || depth <= 0 || !out) return GN_OK;
  Dev::ScoreLevel &L = d.lv[2 - depth];
  HIP_TRY(L.sel.ensure(n + 1));
  HIP_TRY(L.pos.ensure(n + 1));
  HIP_TRY(launch_score_select(out, n, L.sel.p, s));
  HIP_TRY(exclusive_scan_u64(L.sel.p, L.pos.p, n + 1, d.scan_tmp, d.scan_bytes, s));
  uint64_t m = 0;
  HIP_TRY(hipMemcpyAsync(&m, L.pos.p + n, sizeof(m), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (!m) return GN_OK;
  HIP_TRY(L.idx.ensure(m));
  HIP_TRY(L.boards.ensure(m));
  HIP_TRY(L.counts.ensure(m + 1));
  HIP_TRY(L.offsets.ensure(m + 1));
  HIP_TRY(launch_score_gather(boards, L.sel.p, L.pos.p, n, L.idx.p, L.boards.p, s));
  if (replies) {
    uint64_t t = 0;
    HIP_TRY(launch_score_replies(L.idx.p, m, d.offsets.p, L.counts.p, L.offsets.p, d.scan_tmp, d.scan_bytes, &t, s));
    HIP_TRY(L.moves.ensure(std::max<uint64_t>(t, 1)));
    HIP_TRY(L.children.ensure(std::max<uint64_t>(t, 1)));
    HIP_TRY(L.ce.ensure(std::max<uint64_t>(t, 1)));
    HIP_TRY(L.sv.ensure(std::max<uint64_t>(t, 1)));
    HIP_TRY(launch_score_replies_fill(L.idx.p, m, d.offsets.p, L.offsets.p, replies->rec, replies->moves, d.unpacked.p,
                                      d.tables, L.ce.p, L.children.p, L.moves.p, s));
    int rc = resolve_scores(ctx, d, L.children.p, t, mode, L.ce.p, L.sv.p, s, depth - 1);
    if (rc) return rc;
    HIP_TRY(launch_score_reduce(L.boards.p, m, L.idx.p, L.offsets.p, L.moves.p, L.ce.p, L.sv.p, ctx->P, out, sv_out,
                                s));
    return GN_OK;
  }
  HIP_TRY(hipMemsetAsync(L.counts.p + m, 0, sizeof(uint64_t), s));
  HIP_TRY(launch_count_children(L.boards.p, m, d.tables, L.counts.p, s));
  HIP_TRY(exclusive_scan_u64(L.counts.p, L.offsets.p, m + 1, d.scan_tmp, d.scan_bytes, s));
  uint64_t t = 0;
  HIP_TRY(hipMemcpyAsync(&t, L.offsets.p + m, sizeof(t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  HIP_TRY(L.moves.ensure(std::max<uint64_t>(t, 1)));
  HIP_TRY(L.owner.ensure(std::max<uint64_t>(t, 1)));
  HIP_TRY(L.children.ensure(std::max<uint64_t>(t, 1)));
  HIP_TRY(L.ce.ensure(std::max<uint64_t>(t, 1)));
  HIP_TRY(L.sv.ensure(std::max<uint64_t>(t, 1)));
  HIP_TRY(launch_write_children(L.boards.p, m, d.tables, L.offsets.p, 0, t, L.children.p, L.moves.p, L.owner.p,
                                nullptr, nullptr, 1, nullptr, s));
  int rc = evaluate_on(ctx, d, L.children.p, t, mode, L.ce.p, s, nullptr);
  if (rc) return rc;
  if ((rc = resolve_scores(ctx, d, L.children.p, t, mode, L.ce.p, L.sv.p, s, depth - 1)) != GN_OK) return rc;
  HIP_TRY(launch_score_reduce(L.boards.p, m, L.idx.p, L.offsets.p, L.moves.p, L.ce.p, L.sv.p, ctx->P, out, sv_out, s));
  return GN_OK;
}

// ---------------------------------------------------------- sharding -----
// The one partitioner of the library and of bench.py / fishnet_amd/dist.py (through
// gn_partition): contiguous item ranges, cut so that shard k starts at the first item
// whose weight prefix reaches k/n_shards of the total (weights NULL: all 1, i.e. equal
// ranges).  Items are games (weight = positions) or parents (weight 1), so a game is
// never split and each device keeps a game's consecutive parents for the chained walk
// ("contiguous ranges of parents, game-aligned, per GPU"; the
// reference's analog is the worker fan-out, /root/reference/src/main.rs:151-161).
static void partition(const uint32_t *weights, size_t n, int ns, size_t *bounds) {
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += weights ? weights[i] : 1u;
  bounds[0] = 0;
  size_t i = 0;
  uint64_t acc = 0;
  for (int k = 1; k < ns; ++k) {
    const uint64_t target = (total * (uint64_t)k + (uint64_t)ns - 1) / (uint64_t)ns; // ceil(k * total / ns)
    while (i < n && acc < target) acc += weights ? weights[i++] : (++i, 1u);
    bounds[k] = i;
  }
  bounds[ns] = n;
}

// Runs f(k) for every device k on its own host thread (one device: inline) with that
// device's lock held; returns the first failing code with its message.
template <class F>
static int for_each_device(gn_ctx *ctx, F &&f) {
  const size_t nd = ctx->devs.size();
  std::vector<int> rcs(nd, GN_OK);
  std::vector<std::string> errs(nd);
  auto work = [&](size_t k) {
    Dev &d = *ctx->devs[k];
    std::lock_guard<std::mutex> lk(d.mu);
    rcs[k] = f(k, d);
    if (rcs[k]) errs[k] = g_err;
  };
  if (nd == 1) work(0);
  else {
    std::vector<std::thread> th;
    for (size_t k = 0; k < nd; ++k) th.emplace_back(work, k);
    for (auto &t : th) t.join();
  }
  for (size_t k = 0; k < nd; ++k)
    if (rcs[k]) {
      g_err = errs[k];
      return rcs[k];
    }
  return GN_OK;
}

// A FastBatch for nb positions in mode: buffers, pinned staging, the captured graph (d.mu held).
static int fast_build(gn_ctx *ctx, Dev &d, FastBatch &f, size_t nb, int mode) {
  // reply capacities: a lichess game has ~4 % of its positions in check with ~4 replies each (a
  // 128-position class: ~12 replies against 320); the evaluation is sized by the capacities, so a
  // smaller one is cheaper, and a batch beyond them reruns on the general path
  f.nb = nb, f.c1 = nb / 2 + 256, f.c2 = nb / 4 + 256, f.mode = mode, f.gen = ctx->graph_gen.load();
  const size_t na = nb + f.c1 + f.c2;
  HIP_TRY(hipEventCreateWithFlags(&f.done, hipEventDisableTiming));
  HIP_TRY(hipHostMalloc((void **)&f.h_in, nb * sizeof(gn_board), hipHostMallocDefault));
  HIP_TRY(hipHostMalloc((void **)&f.h_out, (nb + 1) * sizeof(gn_eval), hipHostMallocDefault));
  HIP_TRY(f.all.ensure(na));
  HIP_TRY(f.rec.ensure(na + 1));
  f.in = f.all.p, f.r1 = f.in + nb, f.r2 = f.r1 + f.c1;
  f.out = f.rec.p + 1, f.e1 = f.out + nb, f.e2 = f.e1 + f.c1;
  HIP_TRY(f.m1.ensure(f.c1));
  HIP_TRY(f.sv1.ensure(f.c1));
  HIP_TRY(f.m2.ensure(f.c2));
  HIP_TRY(f.sv2.ensure(f.c2));
  HIP_TRY(f.off0.ensure(nb + 1));
  HIP_TRY(f.off1.ensure(f.c1 + 1));
  HIP_TRY(f.eb.osm.ensure(na));
  HIP_TRY(f.eb.obg.ensure(na));
  HIP_TRY(f.eb.nsm.ensure(na));
  HIP_TRY(f.eb.nbg.ensure(na));
  const hipStream_t s = d.stream;
  uint32_t *flag = reinterpret_cast<uint32_t *>(f.rec.p);
  // (round 6: the big net on a graph branch of its own, beside the small net, measured slower --
  // p50 0.200 against 0.180 ms, the join's cross-queue wait costing more than the overlap gave)
  HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  auto seq = [&]() -> int {
    HIP_TRY(hipMemcpyAsync(f.in, f.h_in, nb * sizeof(gn_board), hipMemcpyHostToDevice, s));
    // level 1: the replies of the in-check positions; level 2: those of the replies in check --
    // both from the boards alone (the selection is board properties), so that one evaluation
    // then covers the three levels (round 6: three evaluations, one per level, nine launches)
    HIP_TRY(launch_reply_level(f.in, nb, d.tables, f.off0.p, f.c1, f.r1, f.m1.p, flag, 1, s));
    HIP_TRY(launch_reply_level(f.r1, f.c1, d.tables, f.off1.p, f.c2, f.r2, f.m2.p, flag, 0, s));
    int rc = evaluate_on(ctx, d, f.all.p, na, mode, f.out, s, nullptr, nullptr, 1, nullptr, &f.eb, false);
    if (rc) return rc;
#ifndef GN_AB_FAST_TWO_REDUCES // A/B: the two reductions as two launches
    HIP_TRY(launch_score_reduce2(f.r1, f.c1, f.off1.p, f.m2.p, f.e2, f.sv2.p, f.e1, f.sv1.p, f.in, nb, f.off0.p, f.m1.p,
                                 ctx->P, f.out, s));
#else
    HIP_TRY(launch_score_reduce(f.r1, f.c1, nullptr, f.off1.p, f.m2.p, f.e2, f.sv2.p, ctx->P, f.e1, f.sv1.p, s));
    HIP_TRY(launch_score_reduce(f.in, nb, nullptr, f.off0.p, f.m1.p, f.e1, f.sv1.p, ctx->P, f.out, nullptr, s));
#endif
    HIP_TRY(hipMemcpyAsync(f.h_out, f.rec.p, (nb + 1) * sizeof(gn_eval), hipMemcpyDeviceToHost, s));
    return GN_OK;
  };
  const int rc = seq();
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(s, &g);
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  HIP_TRY(ec);
  f.graph = g;
  HIP_TRY(hipGraphInstantiate(&f.exec, f.graph, nullptr, nullptr, 0));
  return GN_OK;
}

// One small batch through its graph (one device; lk holds d.mu, released while the launch runs).
// *done = false: a reply level overflowed and nothing was written (the caller runs the general
// path).  With both instances of the class in flight, the call waits for one.
static int fast_run(gn_ctx *ctx, Dev &d, std::unique_lock<std::mutex> &lk, const gn_board *boards, size_t n, int mode,
                    gn_eval *out, bool *done) {
  *done = false;
  size_t nb = FAST_NB0;
  int k = 0;
  while (nb < n) nb <<= 1, ++k;
  auto &inst = d.fast[k][mode];
  auto busy = [&](int i) { return inst[i] && inst[i]->busy; };
  while (busy(0) && busy(1)) d.fast_cv.wait(lk);
  std::unique_ptr<FastBatch> &fp = inst[busy(0) ? 1 : 0];
  HIP_TRY(hipSetDevice(d.id));
  if (!fp || fp->gen != ctx->graph_gen.load()) {
    if (fp) HIP_TRY(hipEventSynchronize(fp->done)); // (its last launch is done: the call waited for it)
    fp.reset(new FastBatch());
    const int rc = fast_build(ctx, d, *fp, nb, mode);
    if (rc) {
      fp.reset();
      return rc;
    }
  }
  FastBatch &f = *fp;
  memcpy(f.h_in, boards, n * sizeof(gn_board));
  if (nb > n) memset(f.h_in + n, 0, (nb - n) * sizeof(gn_board));
  {
    SeqGuard sg(d, d.stream);
    HIP_TRY(sg.e);
    HIP_TRY(hipGraphLaunch(f.exec, d.stream));
    HIP_TRY(hipEventRecord(f.done, d.stream));
  }
  // wait without the device's lock: another call's launch queues behind this one meanwhile
  f.busy = true;
  lk.unlock();
  const hipError_t e = hipEventSynchronize(f.done);
  uint32_t flag = 1;
  if (e == hipSuccess) {
    memcpy(&flag, f.h_out, sizeof(flag));
    if (!flag) memcpy(out, f.h_out + 1, n * sizeof(gn_eval));
  }
  lk.lock();
  f.busy = false;
  d.fast_cv.notify_all();
  HIP_TRY(e);
  ++ctx->fast_runs;
  if (flag) {
    ++ctx->fast_fallbacks;
    return GN_OK;
  }
  *done = true;
  return GN_OK;
}

// Host boards -> device(s) -> gn_eval: contiguous shards, one host thread per device.
static int evaluate_boards_host(gn_ctx *ctx, const gn_board *boards, size_t n, int mode, gn_eval *out) {
  if (!n) return GN_OK;
  if (ctx->fast_batch && n <= FAST_MAX && ctx->devs.size() == 1 && mode >= GN_MODE_FULL && mode <= GN_MODE_SMALL) {
    Dev &d = *ctx->devs[0];
    std::unique_lock<std::mutex> lk(d.mu);
    bool done = false;
    int rc;
    try {
      rc = fast_run(ctx, d, lk, boards, n, mode, out, &done);
    } catch (const std::bad_alloc &) {
      rc = fail(GN_E_NOMEM, "host allocation failed");
    }
    if (rc || done) return rc;
  }
  try {
    std::vector<size_t> b(ctx->devs.size() + 1);
    partition(nullptr, n, (int)ctx->devs.size(), b.data());
    return for_each_device(ctx, [&](size_t k, Dev &d) -> int {
      const size_t lo = b[k], hi = b[k + 1];
      if (lo >= hi) return GN_OK;
      HIP_TRY(hipSetDevice(d.id));
      SeqGuard sg(d, d.stream);
      HIP_TRY(sg.e);
      HIP_TRY(d.io_boards.ensure(hi - lo));
      HIP_TRY(d.io_out.ensure(hi - lo));
      HIP_TRY(hipMemcpyAsync(d.io_boards.p, boards + lo, (hi - lo) * sizeof(gn_board), hipMemcpyHostToDevice,
                             d.stream));
      int r = evaluate_on(ctx, d, d.io_boards.p, hi - lo, mode, d.io_out.p, d.stream, nullptr);
      if (!r) r = resolve_scores(ctx, d, d.io_boards.p, hi - lo, mode, d.io_out.p, nullptr, d.stream);
      if (r) return r;
      HIP_TRY(hipMemcpyAsync(out + lo, d.io_out.p, (hi - lo) * sizeof(gn_eval), hipMemcpyDeviceToHost, d.stream));
      HIP_TRY(hipStreamSynchronize(d.stream));
      return GN_OK;
    });
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

// Concurrent gn_evaluate_batch calls merged into one launch (group commit): a call queues
// itself; when no launch is running it leads one over every queued call of its mode (its own
// included), and the calls that queue meanwhile form the next launch.  A lone caller leads at
// once, so nothing waits on a timer.  fishnet's worker pool calls the evaluator once per chunk
// from N workers (/root/reference/src/main.rs:151-161, 263-343), so under load N small calls
// share one set of kernel launches and host round trips instead of N serialised ones.
// Results are those of separate calls (positions are independent).
static int evaluate_coalesced(gn_ctx *ctx, const gn_board *boards, size_t n, int mode, gn_eval *out) {
  if (!ctx->coalesce) return evaluate_boards_host(ctx, boards, n, mode, out);
  auto &C = ctx->co;
  BatchReq me{boards, n, mode, out};
  std::unique_lock<std::mutex> lk(C.mu);
  try {
    C.q.push_back(&me);
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  }
  // every exit (an exception included) takes this call's request off the queue, so that no
  // later leader touches it after this stack frame is gone
  struct Dequeue {
    decltype(C) &c;
    BatchReq *me;
    ~Dequeue() {
      for (size_t i = 0; i < c.q.size(); ++i)
        if (c.q[i] == me) {
          c.q.erase(c.q.begin() + (ptrdiff_t)i);
          break;
        }
    }
  } dq{C, &me};
  while (!me.done) {
    if (me.taken || C.active >= MAX_LEADERS) {
      C.cv.wait(lk);
      continue;
    }
    // the queue is split before the context is marked busy: an allocation failure here leaves
    // the context free and this call off the queue (Dequeue)
    std::vector<BatchReq *> mine, rest;
    try {
      mine.reserve(C.q.size()), rest.reserve(C.q.size());
    } catch (const std::bad_alloc &) {
      return fail(GN_E_NOMEM, "host allocation failed");
    }
    for (BatchReq *r : C.q) (r->mode == mode ? mine : rest).push_back(r);
    C.q.swap(rest);
    for (BatchReq *r : mine) r->taken = true;
    ++C.active;
    lk.unlock();
    // from here to the re-lock nothing may throw outside the try block: this launch is counted in
    // C.active and only this thread takes it out
    int rc = GN_OK;
    char err[256] = "";
    try {
      if (mine.size() == 1) { // (this call's own request: it was queued and not taken)
        rc = evaluate_boards_host(ctx, mine[0]->boards, mine[0]->n, mode, mine[0]->out);
      } else {
        size_t tot = 0;
        for (BatchReq *r : mine) tot += r->n;
        std::vector<gn_board> all(tot);
        std::vector<gn_eval> res(tot);
        size_t at = 0;
        for (BatchReq *r : mine) std::copy(r->boards, r->boards + r->n, all.begin() + at), at += r->n;
        rc = evaluate_boards_host(ctx, all.data(), tot, mode, res.data());
        at = 0;
        if (rc == GN_OK)
          for (BatchReq *r : mine) std::copy(res.begin() + at, res.begin() + at + r->n, r->out), at += r->n;
      }
    } catch (const std::bad_alloc &) {
      rc = fail(GN_E_NOMEM, "host allocation failed");
    } catch (...) {
      rc = fail(GN_E_INVALID, "unexpected exception");
    }
    if (rc) snprintf(err, sizeof err, "%s", g_err.c_str());
    lk.lock();
    for (BatchReq *r : mine) r->rc = rc, memcpy(r->err, err, sizeof err), r->done = true;
    ++C.launches, C.calls += mine.size();
    --C.active;
    C.cv.notify_all();
  }
  const int rc = me.rc;
  if (rc) {
    try {
      g_err = me.err;
    } catch (...) {
    }
  }
  return rc;
}

// ------------------------------------------------------ host pipeline ----
// The host-buffer expansion (gn_expand_and_evaluate, gn_evaluate_games with children),
// sharded over the context's devices: shard k's parents are resident on its device (uploaded
// boards, or the lichess replay's output); pass 1 counts every shard's children so that each
// shard knows where its children go in the caller's arrays; pass 2 expands a shard in chunks
// of whole games, and a drain thread downloads chunk c's records on the device's copy
// stream while chunk c + 1 computes (two slots of device output buffers).
using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t).count();
}

// f(k, d, lo, hi) on every device k whose shard [b[k], b[k + 1]) is not empty, one host thread
// per device (the caller holds every device lock); the first failure's code and message.
template <class F>
static int run_shards(gn_ctx *ctx, const std::vector<size_t> &b, F &&f) {
  const size_t nd = ctx->devs.size();
  std::vector<int> rcs(nd, GN_OK);
  std::vector<std::string> errs(nd);
  auto work = [&](size_t k) {
    if (b[k] >= b[k + 1]) return;
    try {
      rcs[k] = f(k, *ctx->devs[k], b[k], b[k + 1]);
    } catch (const std::bad_alloc &) {
      rcs[k] = fail(GN_E_NOMEM, "host allocation failed");
    } catch (...) {
      rcs[k] = fail(GN_E_INVALID, "unexpected exception");
    }
    if (rcs[k]) errs[k] = g_err;
  };
  if (nd == 1) work(0);
  else {
    std::vector<std::thread> th;
    for (size_t k = 0; k < nd; ++k) th.emplace_back(work, k);
    for (auto &t : th) t.join();
  }
  for (size_t k = 0; k < nd; ++k)
    if (rcs[k]) {
      g_err = errs[k];
      return rcs[k];
    }
  return GN_OK;
}

static void reset_host_stats(gn_ctx *ctx) {
  for (auto &dp : ctx->devs) dp->t_upload = dp->t_replay = dp->t_compute = dp->t_download = dp->t_tail = 0;
}

// Chunk bounds of a shard's m parents: cut only where `starts` allows (the first parent of each
// game, ascending; empty: anywhere), each chunk >= target parents; {0, ..., m}.
static std::vector<size_t> chunk_bounds(size_t m, const std::vector<size_t> &starts, size_t target) {
  std::vector<size_t> c{0};
  size_t j = 0;
  while (c.back() < m) {
    const size_t want = c.back() + std::max<size_t>(target, 1);
    if (want >= m) break;
    if (starts.empty()) {
      c.push_back(want);
      continue;
    }
    while (j < starts.size() && starts[j] < want) ++j;
    if (j == starts.size() || starts[j] >= m) break;
    c.push_back(starts[j]);
  }
  c.push_back(m);
  return c;
}

// The chunks of a shard's m parents for the pipeline below, cut only at `starts` (game starts;
// empty: anywhere).  opt > 0 (GN_OPT_CHUNK_PARENTS): chunks of >= opt parents.  Automatic: each
// chunk costs a fixed few ms (the row stream's and the plan's last blocks run on a part-idle
// GPU, and the chunk's launches and syncs), and only the last chunk's download is not
// overlapped, so: a shard below 3 x MIN parents is one chunk (MIN = 2,048 games of 81 parents,
// the least that keeps chain_len's full block length); otherwise a short last chunk of
// max(MIN, m / 8) parents after chunks of <= 2 M parents (round 3 cut eight equal chunks: 35 ms
// of per-chunk tails per 4 M parents).
static std::vector<size_t> chunk_plan(size_t m, const std::vector<size_t> &starts, int64_t opt) {
  if (opt > 0) return chunk_bounds(m, starts, (size_t)opt);
  constexpr size_t MIN = (size_t)2048 * 81, BIG = 2000000;
  if (m < 3 * MIN) return {0, m};
  const size_t last = std::max(MIN, m / 8), rest = m - last, k = (rest + BIG - 1) / BIG;
  std::vector<size_t> c{0};
  for (size_t i = 1; i <= k; ++i) {
    size_t x = rest * i / k; // a cut wanted here, moved to the next game start
    if (!starts.empty()) {
      auto it = std::lower_bound(starts.begin(), starts.end(), x);
      x = it == starts.end() ? m : *it;
    }
    if (x > c.back() && x < m) c.push_back(x);
  }
  c.push_back(m);
  return c;
}

// Pass 1 of a shard: its m device-resident parents' child offsets (m + 1, relative) to the host.
static int count_shard(Dev &d, const gn_board *d_par, size_t m, std::vector<uint64_t> &off) {
  size_t total = 0;
  HIP_TRY(count_children(d, d_par, m, d.stream, &total));
  off.resize(m + 1);
  HIP_TRY(hipMemcpy(off.data(), d.offsets.p, (m + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return GN_OK;
}

// Pass 2 of a shard (see above).  off: the shard's child offsets from pass 1; results to
// parent_out[0, m) (optional), child_moves / child_out[0, off[m]) (the caller's arrays at this
// shard's base).
static int expand_pipelined(gn_ctx *ctx, Dev &d, const gn_board *d_par, size_t m, int mode,
                            const std::vector<uint64_t> &off, const std::vector<size_t> &chunks, gn_eval *parent_out,
                            uint16_t *child_moves, gn_child *child_out) {
  hipStream_t s = d.stream;
  size_t maxp = 1, maxc = 1;
  for (size_t c = 0; c + 1 < chunks.size(); ++c)
    maxp = std::max(maxp, chunks[c + 1] - chunks[c]),
    maxc = std::max<size_t>(maxc, off[chunks[c + 1]] - off[chunks[c]]);
  for (int k = 0; k < 2; ++k) {
    HIP_TRY(d.po2[k].ensure(maxp));
    HIP_TRY(d.co2[k].ensure(maxc));
    HIP_TRY(d.cc2[k].ensure(maxc));
    HIP_TRY(d.mv2[k].ensure(maxc));
  }
  int drc[2] = {GN_OK, GN_OK};
  std::string derr[2];
  double dms[2] = {0, 0};
  std::thread drain[2];
  struct Joiner { // joins the drain threads on every way out (an exception included), before
    std::thread *t; // the state they write goes out of scope
    ~Joiner() {
      for (int i = 0; i < 2; ++i)
        if (t[i].joinable()) t[i].join();
    }
  } joiner{drain};
  auto join = [&](int k) -> int {
    if (drain[k].joinable()) drain[k].join();
    d.t_download += dms[k], dms[k] = 0;
    if (!drc[k]) return GN_OK;
    const int r = drc[k];
    drc[k] = GN_OK;
    g_err = derr[k];
    return r;
  };
  int rc = GN_OK;
  auto drain_chunk = [&](int k, size_t pa, size_t mp, size_t t, uint64_t cb) {
    drain[k] = std::thread([&, k, pa, mp, t, cb] {
      const auto t1 = Clock::now();
      hipError_t e = hipSetDevice(d.id);
      if (e == hipSuccess) e = hipStreamWaitEvent(d.copy, d.cev[k], 0);
      if (e == hipSuccess && t)
        e = hipMemcpyAsync(child_out + cb, d.cc2[k].p, t * sizeof(gn_child), hipMemcpyDeviceToHost, d.copy);
      if (e == hipSuccess && t)
        e = hipMemcpyAsync(child_moves + cb, d.mv2[k].p, t * sizeof(uint16_t), hipMemcpyDeviceToHost, d.copy);
      if (e == hipSuccess && parent_out)
        e = hipMemcpyAsync(parent_out + pa, d.po2[k].p, mp * sizeof(gn_eval), hipMemcpyDeviceToHost, d.copy);
      if (e == hipSuccess) e = hipStreamSynchronize(d.copy);
      if (e != hipSuccess) drc[k] = GN_E_HIP, derr[k] = std::string("result download failed: ") + hipGetErrorString(e);
      dms[k] = ms_since(t1);
    });
  };
  // GN_OPT_EXPAND_PIPELINE: chunk c + 1's child generation and plan run on the second stream (in
  // the other buffer set) while chunk c's finalize and score rule run
  const bool pipe = ctx->pipeline && plan_path(ctx, d, mode) && ctx->incremental && chunks.size() > 2;
  if (pipe) {
    hipStream_t B = d.front;
    auto front = [&](size_t c) -> int {
      const int k = (int)(c & 1);
      const size_t pa = chunks[c], mp = chunks[c + 1] - pa;
      const uint64_t tc = off[chunks[c + 1]] - off[pa];
      size_t t = 0;
      int r = generate_children(d, d_par + pa, mp, nullptr, d.mv2[k].cap, d.mv2[k].p, true, &t, B, nullptr, nullptr,
                                chain_len(ctx, d, mp), true, mode == GN_MODE_BIG);
      if (!r && t != tc) r = fail(GN_E_HIP, "child count changed between passes (%zu != %zu)", t, (size_t)tc);
      if (!r)
        r = expand_evaluate(ctx, d, d_par + pa, mp, d.frontier[1].p, t, mode, nullptr, nullptr, B, nullptr, nullptr,
                            true, EXP_FRONT);
      if (!r && hipEventRecord(d.ev_planned, B) != hipSuccess) r = fail(GN_E_HIP, "hipEventRecord failed");
      return r;
    };
    // the front starts after what the device stream holds (the parents' upload / replay)
    if (hipEventRecord(d.ev_streamed, s) != hipSuccess || hipStreamWaitEvent(B, d.ev_streamed, 0) != hipSuccess)
      return fail(GN_E_HIP, "hipStreamWaitEvent failed");
    // the partial sums sized for the largest chunk now: a later front runs beside a back half that
    // reads them and may not reallocate them (part_locked)
    if (d.has[BIG] && d.net[BIG].L1 == 3072 && ctx->stream_slices == 3 &&
        d.part.ensure((size_t)GN_PART_SLICES * 16 * (maxp + maxc)) != hipSuccess)
      (void)hipGetLastError(); // (then the chunks that do not fit stream whole rows)
    d.part_locked = true;
    struct Unlock {
      Dev &d;
      ~Unlock() { d.part_locked = false; }
    } unlock{d};
    rc = front(0);
    for (size_t c = 0; c + 1 < chunks.size() && rc == GN_OK; ++c) {
      const int k = (int)(c & 1);
      const size_t pa = chunks[c], mp = chunks[c + 1] - pa;
      const uint64_t cb = off[pa], t = off[chunks[c + 1]] - cb;
      const auto t0 = Clock::now();
      if (hipStreamWaitEvent(s, d.ev_planned, 0) != hipSuccess) {
        rc = fail(GN_E_HIP, "hipStreamWaitEvent failed");
        break;
      }
      rc = expand_evaluate(ctx, d, d_par + pa, mp, d.frontier[1].p, t, mode, d.po2[k].p, d.co2[k].p, s, nullptr,
                           nullptr, true, EXP_BACK, d.ev_streamed);
      if (rc) break;
      const bool more = c + 2 < chunks.size();
      if (more) { // the next chunk's front (slot k ^ 1: its previous chunk downloaded first)
        if ((rc = join(k ^ 1)) != GN_OK) break;
        swap_sets(d);
        if (ctx->pipeline != 2 && hipStreamWaitEvent(B, d.ev_streamed, 0) != hipSuccess)
          rc = fail(GN_E_HIP, "hipStreamWaitEvent failed");
        if (!rc) rc = front(c + 1);
        swap_sets(d);
        if (rc) break;
      }
      const Replies rp{d.co2[k].p, d.mv2[k].p};
      rc = resolve_scores(ctx, d, d_par + pa, mp, mode, d.po2[k].p, nullptr, s, 2, &rp);
      if (!rc && launch_pack_children(d.co2[k].p, t, d.cc2[k].p, s) != hipSuccess)
        rc = fail(GN_E_HIP, "child record packing failed");
      if (!rc) rc = check_plan(d, s); // synchronises the stream: chunk c is computed
      if (rc) break;
      d.t_compute += ms_since(t0);
      if (hipEventRecord(d.cev[k], s) != hipSuccess) {
        rc = fail(GN_E_HIP, "hipEventRecord failed");
        break;
      }
      drain_chunk(k, pa, mp, t, cb);
      if (more) swap_sets(d);
    }
    if (rc) (void)hipStreamSynchronize(B); // (nothing of a failed call's front may still run)
  }
  for (size_t c = 0; !pipe && c + 1 < chunks.size() && rc == GN_OK; ++c) {
    const int k = (int)(c & 1);
    if ((rc = join(k)) != GN_OK) break; // the slot's previous chunk is downloaded
    const size_t pa = chunks[c], mp = chunks[c + 1] - pa;
    const uint64_t cb = off[pa], tc = off[chunks[c + 1]] - cb;
    const auto t0 = Clock::now();
    size_t t = 0;
    rc = generate_children(d, d_par + pa, mp, nullptr, d.mv2[k].cap, d.mv2[k].p, ctx->incremental, &t, s, nullptr,
                           nullptr, chain_len(ctx, d, mp), plan_path(ctx, d, mode), mode == GN_MODE_BIG);
    if (!rc && t != tc) rc = fail(GN_E_HIP, "child count changed between passes (%zu != %zu)", t, (size_t)tc);
    if (!rc)
      rc = expand_evaluate(ctx, d, d_par + pa, mp, d.frontier[1].p, t, mode, d.po2[k].p, d.co2[k].p, s, nullptr);
    const Replies rp{d.co2[k].p, d.mv2[k].p};
    if (!rc) rc = resolve_scores(ctx, d, d_par + pa, mp, mode, d.po2[k].p, nullptr, s, 2, &rp);
    if (!rc && launch_pack_children(d.co2[k].p, t, d.cc2[k].p, s) != hipSuccess)
      rc = fail(GN_E_HIP, "child record packing failed");
    if (!rc) rc = check_plan(d, s); // synchronises the stream: chunk c is computed
    if (rc) break;
    d.t_compute += ms_since(t0);
    if (hipEventRecord(d.cev[k], s) != hipSuccess) {
      rc = fail(GN_E_HIP, "hipEventRecord failed");
      break;
    }
    drain_chunk(k, pa, mp, t, cb);
  }
  const auto tt = Clock::now();
  for (int k = 0; k < 2; ++k) {
    const int r = join(k);
    if (!rc) rc = r;
  }
  d.t_tail = ms_since(tt);
  return rc;
}

// Host parent boards -> every legal child -> parent/child gn_eval (gn_expand_and_evaluate),
// sharded over every device of the context (equal parent ranges).
static int expand_boards_host(gn_ctx *ctx, const gn_board *boards, size_t n, int mode, gn_eval *parent_out,
                              uint32_t *child_offsets, uint16_t *child_moves, gn_child *child_out, size_t cap) {
  if (!slot(ctx, 0)) return fail(GN_E_INVALID, "bad context");
  if (!n) {
    child_offsets[0] = 0;
    return GN_OK;
  }
  try {
    const size_t nd = ctx->devs.size();
    std::vector<size_t> b(nd + 1);
    partition(nullptr, n, (int)nd, b.data());
    std::vector<std::unique_lock<std::mutex>> locks; // every device lock for the whole call
    for (auto &dp : ctx->devs) locks.emplace_back(dp->mu);
    std::vector<std::vector<uint64_t>> off(nd);
    // pass 1: upload + child counts
    int rc = run_shards(ctx, b, [&](size_t k, Dev &d, size_t lo, size_t hi) -> int {
      HIP_TRY(hipSetDevice(d.id));
      SeqGuard sg(d, d.stream);
      HIP_TRY(sg.e);
      const auto t0 = Clock::now();
      HIP_TRY(d.par.ensure(hi - lo));
      HIP_TRY(hipMemcpyAsync(d.par.p, boards + lo, (hi - lo) * sizeof(gn_board), hipMemcpyHostToDevice, d.stream));
      HIP_TRY(hipStreamSynchronize(d.stream));
      d.t_upload += ms_since(t0);
      return count_shard(d, d.par.p, hi - lo, off[k]);
    });
    if (rc) return rc;
    std::vector<uint64_t> base(nd + 1, 0);
    for (size_t k = 0; k < nd; ++k) base[k + 1] = base[k] + (b[k] < b[k + 1] ? off[k].back() : 0);
    const uint64_t total = base[nd];
    if (total > 0xFFFFFFFFull) return fail(GN_E_CAPACITY, "children exceed 32-bit offsets");
    for (size_t k = 0; k < nd; ++k)
      for (size_t i = b[k]; i < b[k + 1]; ++i) child_offsets[i] = (uint32_t)(base[k] + off[k][i - b[k]]);
    child_offsets[n] = (uint32_t)total;
    if (total > cap) return fail(GN_E_CAPACITY, "%zu children exceed capacity %zu", (size_t)total, cap);
    if (total && (!child_moves || !child_out)) return fail(GN_E_INVALID, "NULL child buffer");
    // pass 2: chunks of 81 parents' multiples (a FEN batch has no games: blocks of 81 = chain_len)
    return run_shards(ctx, b, [&](size_t k, Dev &d, size_t lo, size_t hi) -> int {
      HIP_TRY(hipSetDevice(d.id));
      SeqGuard sg(d, d.stream);
      HIP_TRY(sg.e);
      const size_t m = hi - lo;
      std::vector<size_t> starts;
      for (size_t i = 81; i < m; i += 81) starts.push_back(i);
      return expand_pipelined(ctx, d, d.par.p, m, mode, off[k], chunk_plan(m, starts, ctx->chunk_parents),
                              parent_out ? parent_out + lo : nullptr, child_moves + base[k], child_out + base[k]);
    });
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

// ------------------------------------------------- lichess batch replay ----
// IncomingBatch::from_acquired (/root/reference/src/queue.rs:548-700) for the
// GPU path.  The root FEN is set up with Chess960 castling, ignoring an invalid
// en-passant square or castling right (queue.rs:554-560).  Every UCI move of
// AcquireResponseBody.moves (/root/reference/src/api.rs:306-321) is resolved as
// shakmaty 0.27.3's UciMove::to_move resolves it (queue.rs:576) and played
// (queue.rs:578).  That gives positions 0..=len, position i being the root after
// i moves (queue.rs:605-637); skipPositions marks the ones not analysed
// (queue.rs:617, 633).  A move that does not resolve to a legal move fails the
// game, as `uci.to_move(&pos)?` fails the whole batch in the reference.

// (shakmaty 0.27.3 UciMove::to_move: resolve_uci in chess.h, shared with the GPU replay)
static bool uci_to_move(const Board &B, const char *u, size_t len, uint16_t &out) {
  return resolve_uci(B, host_tables(), uci_code(u, (int)len), out);
}

struct Replay {
  std::vector<gn_board> boards; // positions 0..=len
  std::vector<uint16_t> moves;  // len moves, Stockfish encoding (castling = king takes rook)
  std::vector<uint8_t> skip;    // per position
  int rc = GN_OK;
  std::string err;
};

static void replay_game(const gn_game &g, Replay &r) {
  Board B;
  if (!g.root_fen || !parse_fen(g.root_fen, B)) {
    r.rc = GN_E_INVALID, r.err = "bad root FEN";
    return;
  }
  gn_board pb;
  pack(B, pb);
  r.boards.push_back(pb);
  const char *s = g.uci_moves ? g.uci_moves : "";
  while (*s) {
    while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') ++s;
    if (!*s) break;
    const char *e = s;
    while (*e && *e != ' ' && *e != '\t' && *e != '\n' && *e != '\r') ++e;
    uint16_t m = 0;
    if (!uci_to_move(B, s, (size_t)(e - s), m)) {
      char buf[96];
      snprintf(buf, sizeof(buf), "move %zu (%.*s) is not legal", r.moves.size() + 1, (int)std::min<ptrdiff_t>(e - s, 16), s);
      r.rc = GN_E_ILLEGAL_MOVE, r.err = buf;
      r.boards.clear(), r.moves.clear();
      return;
    }
    B = do_move(B, m);
    pack(B, pb);
    r.boards.push_back(pb);
    r.moves.push_back(m);
    s = e;
  }
  r.skip.assign(r.boards.size(), 0);
  for (size_t k = 0; k < g.n_skip; ++k)
    if (g.skip_positions && g.skip_positions[k] < r.skip.size()) r.skip[g.skip_positions[k]] = 1;
}

// A game prepared on the host for the GPU replay: its root (Position::set on the root FEN)
// and its move tokens as uci_code values (the wire form, whitespace-separated).
struct GamePrep {
  gn_board root;
  bool ok = false;
  std::vector<uint16_t> codes;
};

static void prep_game(const gn_game &g, GamePrep &p) {
  Board B;
  if (!g.root_fen || !parse_fen(g.root_fen, B)) return;
  pack(B, p.root);
  p.ok = true;
  const char *s = g.uci_moves ? g.uci_moves : "";
  while (*s) {
    while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') ++s;
    if (!*s) break;
    const char *e = s;
    while (*e && *e != ' ' && *e != '\t' && *e != '\n' && *e != '\r') ++e;
    p.codes.push_back(uci_code(s, (int)std::min<ptrdiff_t>(e - s, 6)) );
    s = e;
  }
}

// the text of a game's move k (1-based), for the error message (at most 16 characters)
static std::string move_token(const gn_game &g, size_t k) {
  const char *s = g.uci_moves ? g.uci_moves : "";
  for (size_t i = 1; *s; ++i) {
    while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') ++s;
    if (!*s) break;
    const char *e = s;
    while (*e && *e != ' ' && *e != '\t' && *e != '\n' && *e != '\r') ++e;
    if (i == k) return std::string(s, (size_t)std::min<ptrdiff_t>(e - s, 16));
    s = e;
  }
  return "";
}

// ============================================================ C-ABI ========
extern "C" {

int gn_replay_game(const gn_game *game, gn_board *positions, uint8_t *skipped, uint16_t *moves, size_t cap,
                   size_t *n_positions) {
  if (!game || !n_positions) return fail(GN_E_INVALID, "NULL argument");
  try {
    Replay r;
    replay_game(*game, r);
    *n_positions = r.boards.size();
    if (r.rc) return fail(r.rc, "%s", r.err.c_str());
    if (r.boards.size() > cap) return fail(GN_E_CAPACITY, "%zu positions exceed capacity %zu", r.boards.size(), cap);
    if (positions) memcpy(positions, r.boards.data(), r.boards.size() * sizeof(gn_board));
    if (skipped) memcpy(skipped, r.skip.data(), r.skip.size());
    if (moves && !r.moves.empty()) memcpy(moves, r.moves.data(), r.moves.size() * sizeof(uint16_t));
    return GN_OK;
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  }
}

int gn_evaluate_games(gn_ctx *ctx, const gn_game *games, size_t n_games, int mode, int with_children,
                      uint32_t *position_offsets, int32_t *game_status, gn_eval *position_out, size_t position_cap,
                      uint32_t *child_offsets, uint16_t *child_moves, gn_child *child_out, size_t child_cap) {
  if (!slot(ctx, 0)) return fail(GN_E_INVALID, "bad context");
  if (n_games && (!games || !position_offsets || !game_status)) return fail(GN_E_INVALID, "NULL argument");
  if (with_children && !child_offsets) return fail(GN_E_INVALID, "child_offsets is NULL");
  if (mode < GN_MODE_FULL || mode > GN_MODE_SMALL) return fail(GN_E_INVALID, "bad mode %d", mode);
  try {
    const auto T0 = Clock::now();
    reset_host_stats(ctx);
    // host: root FENs parsed, UCI moves tokenized (the wire form, AcquireResponseBody.moves)
    std::vector<GamePrep> prep(n_games);
    parallel_for(n_games, 64, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) prep_game(games[i], prep[i]);
    });
    ctx->t_parse = ms_since(T0);
    // games sharded over the devices, never split, weighted by their positions (moves + 1)
    const size_t nd = ctx->devs.size();
    std::vector<uint32_t> w(n_games);
    for (size_t i = 0; i < n_games; ++i) w[i] = prep[i].ok ? (uint32_t)prep[i].codes.size() + 1 : 0;
    std::vector<size_t> gb(nd + 1);
    partition(w.data(), n_games, (int)nd, gb.data());
    std::vector<std::unique_lock<std::mutex>> locks; // every device lock for the whole call
    for (auto &dp : ctx->devs) locks.emplace_back(dp->mu);
    // phase A: each device replays its games (replay_games_kernel) and reports their status
    std::vector<std::vector<size_t>> glist(nd);  // the device's replayed games (global index)
    std::vector<std::vector<uint64_t>> moff(nd); // their move-code offsets
    std::vector<std::vector<int32_t>> st(nd);    // their status (0 or the first illegal move)
    int rc = run_shards(ctx, gb, [&](size_t k, Dev &d, size_t g0, size_t g1) -> int {
      HIP_TRY(hipSetDevice(d.id));
      SeqGuard sg(d, d.stream);
      HIP_TRY(sg.e);
      auto &gl = glist[k];
      auto &mo = moff[k];
      mo.push_back(0);
      for (size_t g = g0; g < g1; ++g)
        if (prep[g].ok) gl.push_back(g), mo.push_back(mo.back() + prep[g].codes.size());
      const size_t ng = gl.size(), nm = mo.back();
      if (!ng) return GN_OK;
      std::vector<uint16_t> codes(std::max<size_t>(nm, 1));
      std::vector<gn_board> roots(ng);
      for (size_t j = 0; j < ng; ++j) {
        roots[j] = prep[gl[j]].root;
        std::copy(prep[gl[j]].codes.begin(), prep[gl[j]].codes.end(), codes.begin() + mo[j]);
      }
      const auto t0 = Clock::now();
      HIP_TRY(d.roots.ensure(ng));
      HIP_TRY(d.moff.ensure(ng + 1));
      HIP_TRY(d.codes.ensure(std::max<size_t>(nm, 1)));
      HIP_TRY(d.rboards.ensure(nm + ng));
      HIP_TRY(d.smoves.ensure(std::max<size_t>(nm, 1)));
      HIP_TRY(d.rstatus.ensure(ng));
      hipStream_t s = d.stream;
      HIP_TRY(hipMemcpyAsync(d.roots.p, roots.data(), ng * sizeof(gn_board), hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(d.moff.p, mo.data(), (ng + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(d.codes.p, codes.data(), codes.size() * sizeof(uint16_t), hipMemcpyHostToDevice, s));
      HIP_TRY(hipStreamSynchronize(s));
      d.t_upload += ms_since(t0);
      const auto t1 = Clock::now();
      HIP_TRY(launch_replay_games(d.roots.p, ng, d.moff.p, d.codes.p, d.tables, d.rboards.p, d.smoves.p, d.rstatus.p, s));
      st[k].resize(ng);
      HIP_TRY(hipMemcpyAsync(st[k].data(), d.rstatus.p, ng * sizeof(int32_t), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      d.t_replay += ms_since(t1);
      return GN_OK;
    });
    if (rc) return rc;
    // host: status, position offsets; the evaluated (non-skipped) positions of each device
    std::vector<int32_t> gst(n_games, GN_OK);
    std::vector<uint32_t> npos(n_games, 0);
    std::string last_err;
    for (size_t k = 0; k < nd; ++k)
      for (size_t j = 0; j < glist[k].size(); ++j) {
        const size_t g = glist[k][j];
        if (st[k][j]) {
          gst[g] = GN_E_ILLEGAL_MOVE;
          last_err = "move " + std::to_string(st[k][j]) + " (" + move_token(games[g], (size_t)st[k][j]) + ") is not legal";
        } else {
          npos[g] = (uint32_t)(moff[k][j + 1] - moff[k][j] + 1);
        }
      }
    uint64_t total = 0;
    for (size_t g = 0; g < n_games; ++g) {
      if (!prep[g].ok) gst[g] = GN_E_INVALID, last_err = "bad root FEN";
      game_status[g] = gst[g];
      position_offsets[g] = (uint32_t)total;
      total += npos[g];
    }
    if (total > 0xFFFFFFFFull) return fail(GN_E_CAPACITY, "positions exceed 32-bit offsets");
    position_offsets[n_games] = (uint32_t)total;
    if (total > position_cap) return fail(GN_E_CAPACITY, "%zu positions exceed capacity %zu", (size_t)total, position_cap);
    if (total && !position_out) return fail(GN_E_INVALID, "position_out is NULL");
    // The evaluated positions of each device.  Fast path (the common case): every game of the
    // device replayed and none has a skipped position, so its positions are the replay's boards
    // as they lie (rboards: game j's position p at moff[j] + j + p) and one contiguous run of
    // position_out from p0[k]: the expansion reads rboards in place and writes the caller's
    // arrays directly.  Otherwise the evaluated positions are gathered (src: board index,
    // where: output index) into contiguous parents and their records scattered back.
    std::vector<std::vector<uint32_t>> src(nd), where(nd);
    std::vector<std::vector<size_t>> starts(nd); // first evaluated position of each game
    std::vector<uint8_t> fast(nd, 0);
    std::vector<size_t> mcount(nd, 0), p0(nd, 0);
    std::vector<uint8_t> skip;
    for (size_t k = 0; k < nd; ++k) {
      bool f = true;
      for (size_t j = 0; j < glist[k].size() && f; ++j) {
        const size_t g = glist[k][j];
        f = st[k][j] == 0;
        for (size_t q = 0; q < games[g].n_skip && f; ++q)
          f = !games[g].skip_positions || games[g].skip_positions[q] >= npos[g];
      }
      if (f) {
        fast[k] = 1;
        mcount[k] = glist[k].empty() ? 0 : (size_t)moff[k].back() + glist[k].size();
        p0[k] = glist[k].empty() ? 0 : position_offsets[glist[k][0]];
        for (size_t j = 0; j < glist[k].size(); ++j) starts[k].push_back((size_t)moff[k][j] + j);
        continue;
      }
      for (size_t j = 0; j < glist[k].size(); ++j) {
        const size_t g = glist[k][j];
        if (!npos[g]) continue;
        skip.assign(npos[g], 0);
        for (size_t q = 0; q < games[g].n_skip; ++q)
          if (games[g].skip_positions && games[g].skip_positions[q] < npos[g]) skip[games[g].skip_positions[q]] = 1;
        starts[k].push_back(src[k].size());
        for (uint32_t p = 0; p < npos[g]; ++p) {
          const size_t at = position_offsets[g] + p;
          if (skip[p]) {
            position_out[at] = gn_eval{0, 0, 0, 0, 0, (uint16_t)(GN_FLAG_SKIPPED | GN_FLAG_NO_SCORE), 0};
          } else {
            src[k].push_back((uint32_t)(moff[k][j] + j + p));
            where[k].push_back((uint32_t)at);
          }
        }
      }
      mcount[k] = src[k].size();
    }
    // phase B: (slow path) the evaluated positions gathered into contiguous parents; evaluated
    // (no children) or counted (pass 1 of the expansion)
    std::vector<std::vector<gn_eval>> res(nd);
    std::vector<std::vector<uint64_t>> off(nd);
    std::vector<size_t> db(nd + 1);
    for (size_t k = 0; k <= nd; ++k) db[k] = k; // one "item" per device: run_shards' shard k = device k
    auto has = [&](size_t k) { return mcount[k] > 0; };
    auto parents_of = [&](size_t k) -> const gn_board * { return fast[k] ? ctx->devs[k]->rboards.p : ctx->devs[k]->par.p; };
    auto records_of = [&](size_t k) -> gn_eval * { return fast[k] ? position_out + p0[k] : res[k].data(); };
    rc = run_shards(ctx, db, [&](size_t k, Dev &d, size_t, size_t) -> int {
      if (!has(k)) return GN_OK;
      HIP_TRY(hipSetDevice(d.id));
      SeqGuard sg(d, d.stream);
      HIP_TRY(sg.e);
      const size_t m = mcount[k];
      hipStream_t s = d.stream;
      if (!fast[k]) {
        const auto t0 = Clock::now();
        HIP_TRY(d.gidx.ensure(m));
        HIP_TRY(d.par.ensure(m));
        HIP_TRY(hipMemcpyAsync(d.gidx.p, src[k].data(), m * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        HIP_TRY(launch_gather_boards(d.rboards.p, d.gidx.p, m, d.par.p, s));
        HIP_TRY(hipStreamSynchronize(s));
        d.t_upload += ms_since(t0);
        res[k].resize(m);
      }
      if (with_children) return count_shard(d, parents_of(k), m, off[k]);
      const auto t1 = Clock::now();
      HIP_TRY(d.io_out.ensure(m));
      int r = evaluate_on(ctx, d, parents_of(k), m, mode, d.io_out.p, s, nullptr);
      if (!r) r = resolve_scores(ctx, d, parents_of(k), m, mode, d.io_out.p, nullptr, s);
      if (r) return r;
      HIP_TRY(hipStreamSynchronize(s));
      d.t_compute += ms_since(t1);
      const auto t2 = Clock::now();
      HIP_TRY(hipMemcpy(records_of(k), d.io_out.p, m * sizeof(gn_eval), hipMemcpyDeviceToHost));
      d.t_download += ms_since(t2);
      return GN_OK;
    });
    if (rc) return rc;
    if (with_children) {
      std::vector<uint64_t> cb(nd + 1, 0);
      for (size_t k = 0; k < nd; ++k) cb[k + 1] = cb[k] + (has(k) ? off[k].back() : 0);
      const uint64_t ctot = cb[nd];
      if (ctot > 0xFFFFFFFFull) return fail(GN_E_CAPACITY, "children exceed 32-bit offsets");
      // child offsets over all positions (skipped ones: no children, the next position's offset)
      const bool all_fast = std::all_of(fast.begin(), fast.end(), [](uint8_t f) { return f != 0; });
      if (!all_fast)
        for (size_t g = 0; g < n_games; ++g)
          for (uint32_t p = 0; p < npos[g]; ++p) child_offsets[position_offsets[g] + p] = 0xFFFFFFFFu;
      for (size_t k = 0; k < nd; ++k) {
        if (!has(k)) continue;
        if (fast[k])
          for (size_t e = 0; e < mcount[k]; ++e) child_offsets[p0[k] + e] = (uint32_t)(cb[k] + off[k][e]);
        else
          for (size_t e = 0; e < where[k].size(); ++e) child_offsets[where[k][e]] = (uint32_t)(cb[k] + off[k][e]);
      }
      if (!all_fast) {
        uint32_t next = (uint32_t)ctot;
        for (size_t at = total; at-- > 0;) {
          if (child_offsets[at] == 0xFFFFFFFFu) child_offsets[at] = next;
          else next = child_offsets[at];
        }
      }
      child_offsets[total] = (uint32_t)ctot;
      if (ctot > child_cap) return fail(GN_E_CAPACITY, "%zu children exceed capacity %zu", (size_t)ctot, child_cap);
      if (ctot && (!child_moves || !child_out)) return fail(GN_E_INVALID, "NULL child buffer");
      // phase C: the expansion pipeline, chunks cut at game starts
      rc = run_shards(ctx, db, [&](size_t k, Dev &d, size_t, size_t) -> int {
        if (!has(k)) return GN_OK;
        HIP_TRY(hipSetDevice(d.id));
        SeqGuard sg(d, d.stream);
        HIP_TRY(sg.e);
        const size_t m = mcount[k];
        return expand_pipelined(ctx, d, parents_of(k), m, mode, off[k], chunk_plan(m, starts[k], ctx->chunk_parents),
                                records_of(k), child_moves + cb[k], child_out + cb[k]);
      });
      if (rc) return rc;
    }
    for (size_t k = 0; k < nd; ++k)
      for (size_t e = 0; e < where[k].size(); ++e) position_out[where[k][e]] = res[k][e];
    ctx->t_total = ms_since(T0);
    if (!last_err.empty()) g_err = last_err;
    return GN_OK;
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

int gn_partition(const uint32_t *weights, size_t n_items, int n_shards, size_t *bounds) {
  if (n_shards <= 0 || !bounds) return fail(GN_E_INVALID, "bad shard count / NULL bounds");
  try {
    partition(weights, n_items, n_shards, bounds);
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
  return GN_OK;
}

int gn_abi_version(void) { return GN_ABI_VERSION; }

const char *gn_last_error(void) { return g_err.c_str(); }

// Stockfish names nets "nn-" + the first 12 hex digits of the file's SHA-256 + ".nnue"
// (checked after download by Stockfish's `make net`, which fishnet's build runs,
// /root/reference/build.rs:318-333).  A file named that way must hash to its name.
static int check_net_name(const char *path, const std::vector<uint8_t> &data) {
  const char *base = strrchr(path, '/');
  base = base ? base + 1 : path;
  if (strlen(base) != 20 || strncmp(base, "nn-", 3) != 0 || strcmp(base + 15, ".nnue") != 0) return GN_OK;
  for (int i = 3; i < 15; ++i)
    if (!((base[i] >= '0' && base[i] <= '9') || (base[i] >= 'a' && base[i] <= 'f'))) return GN_OK;
  Sha256 h;
  h.update(data.data(), data.size());
  char hex[65];
  h.hex(hex);
  if (strncmp(hex, base + 3, 12) != 0)
    return fail(GN_E_FORMAT, "%s: content hashes to nn-%.12s.nnue (corrupt or renamed net)", path, hex);
  return GN_OK;
}

int gn_net_sha256(const uint8_t *data, size_t len, char *hex65) {
  if ((!data && len) || !hex65) return fail(GN_E_INVALID, "NULL argument");
  Sha256 h;
  h.update(data, len);
  h.hex(hex65);
  return GN_OK;
}

int gn_load_net(const char *big_path, const char *small_path, const int *devices, int n_devices, gn_ctx **out) {
  try {
    std::vector<uint8_t> b, s;
    if (big_path && !read_file(big_path, b)) return fail(GN_E_IO, "cannot read %s", big_path);
    if (small_path && !read_file(small_path, s)) return fail(GN_E_IO, "cannot read %s", small_path);
    int rc;
    if (big_path && (rc = check_net_name(big_path, b)) != GN_OK) return rc;
    if (small_path && (rc = check_net_name(small_path, s)) != GN_OK) return rc;
    return create(big_path ? b.data() : nullptr, b.size(), small_path ? s.data() : nullptr, s.size(), devices,
                  n_devices, out);
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

// L1 width of a .nnue image from its header hashes (0: not a supported net)
static int net_l1(const uint8_t *d, size_t n) {
  auto u32 = [&](size_t o) { return (uint32_t)d[o] | (uint32_t)d[o + 1] << 8 | (uint32_t)d[o + 2] << 16 | (uint32_t)d[o + 3] << 24; };
  if (n < 12 || u32(0) != NNUE_VERSION) return 0;
  const size_t dl = u32(8);
  if (12 + dl + 4 > n) return 0;
  const uint32_t hash = u32(4), fth = u32(12 + dl);
  for (int c : {3072, 1024, 128})
    if (ft_hash(c) == fth && (ft_hash(c) ^ arch_hash(c)) == hash) return c;
  return 0;
}

// The members of an assets archive (zstd + ar, archive.h); GN_OK or a failure.
static int read_archive(const char *path, std::vector<uint8_t> &img, std::vector<archive::Member> &mem) {
  std::vector<uint8_t> file;
  if (!path || !read_file(path, file)) return fail(GN_E_IO, "cannot read %s", path ? path : "(null)");
  std::string err;
  if (!archive::load_image(file, img, err) || !archive::ar_members(img.data(), img.size(), mem, err))
    return fail(GN_E_FORMAT, "%s: %s", path, err.c_str());
  return GN_OK;
}

int gn_archive_read(const char *path, const char *member, uint8_t *buf, size_t cap, size_t *size) {
  try {
    if (!member || !size) return fail(GN_E_INVALID, "bad argument");
    std::vector<uint8_t> img;
    std::vector<archive::Member> mem;
    int rc = read_archive(path, img, mem);
    if (rc) return rc;
    for (const auto &m : mem)
      if (m.name == member) {
        *size = m.size;
        if (m.size > cap || (!buf && m.size)) return fail(GN_E_CAPACITY, "%s is %zu bytes", member, m.size);
        if (m.size) memcpy(buf, img.data() + m.off, m.size);
        return GN_OK;
      }
    return fail(GN_E_IO, "%s has no member %s", path, member);
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

int gn_load_net_archive(const char *path, const char *big_member, const char *small_member, const int *devices,
                        int n_devices, gn_ctx **out) {
  try {
    std::vector<uint8_t> img;
    std::vector<archive::Member> mem;
    int rc = read_archive(path, img, mem);
    if (rc) return rc;
    const archive::Member *pick[2] = {nullptr, nullptr};
    const char *want[2] = {big_member, small_member};
    for (int w = 0; w < 2; ++w)
      for (const auto &m : mem) {
        const uint8_t *d = img.data() + m.off;
        const int l1 = net_l1(d, m.size);
        const bool ends = m.name.size() > 5 && m.name.compare(m.name.size() - 5, 5, ".nnue") == 0;
        // by name, or the first .nnue of the right kind (big: L1 3072 / 1024, small: 128)
        if (want[w] ? m.name == want[w] : (ends && l1 && ((w == 0) == (l1 != 128)))) {
          pick[w] = &m;
          break;
        }
      }
    if (!pick[0] && !pick[1]) return fail(GN_E_IO, "%s holds no usable .nnue member", path);
    if ((big_member && !pick[0]) || (small_member && !pick[1]))
      return fail(GN_E_IO, "%s has no member %s", path, !pick[0] && big_member ? big_member : small_member);
    for (int w = 0; w < 2; ++w)
      if (pick[w]) { // Stockfish's name check: nn-<first 12 hex of SHA-256>.nnue
        std::vector<uint8_t> data(img.begin() + pick[w]->off, img.begin() + pick[w]->off + pick[w]->size);
        if ((rc = check_net_name(pick[w]->name.c_str(), data)) != GN_OK) return rc;
      }
    return create(pick[0] ? img.data() + pick[0]->off : nullptr, pick[0] ? pick[0]->size : 0,
                  pick[1] ? img.data() + pick[1]->off : nullptr, pick[1] ? pick[1]->size : 0, devices, n_devices,
                  out);
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

int gn_load_net_memory(const uint8_t *big, size_t big_len, const uint8_t *small, size_t small_len, const int *devices,
                       int n_devices, gn_ctx **out) {
  try {
    return create(big, big_len, small, small_len, devices, n_devices, out);
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

void gn_free(gn_ctx *ctx) { destroy(ctx); }

int gn_get_eval_params(const gn_ctx *ctx, gn_eval_params *out) {
  if (!out) return fail(GN_E_INVALID, "out is NULL");
  *out = ctx ? ctx->P : default_params();
  return GN_OK;
}

int gn_set_eval_params(gn_ctx *ctx, const gn_eval_params *p) {
  if (!ctx || !p) return fail(GN_E_INVALID, "NULL argument");
  if (p->material_base == 0 || p->rule50_div == 0 || p->complexity_div_small == 0 || p->complexity_div_big == 0 ||
      p->wdl_material_anchor == 0)
    return fail(GN_E_INVALID, "zero divisor in eval params");
  if (p->wdl_material_min > p->wdl_material_max) return fail(GN_E_INVALID, "wdl material range is empty");
  if ((int64_t)p->wdl_material_max - p->wdl_material_min > 4096) return fail(GN_E_INVALID, "wdl material range too wide");
  if (p->value_clamp < 0 || p->value_clamp >= VALUE_MATE_IN_MAX_PLY)
    return fail(GN_E_INVALID, "value_clamp must be in [0, %d) (static values stay below mate scores)",
                (int)VALUE_MATE_IN_MAX_PLY);
  // to_cp's a(material) >= 1 wherever it is evaluated (every clamped material value), so that
  // |final_cp| <= 100 * value_clamp < 2^23 fits gn_child's 24-bit field (defaults: a ~ 370-400)
  for (int64_t mc = p->wdl_material_min; mc <= (int64_t)p->wdl_material_max; ++mc) { // (int64: max may be INT_MAX)
#pragma clang fp contract(off)
    const double m = (double)mc / (double)p->wdl_material_anchor;
    const double a = ((p->wdl_a[0] * m + p->wdl_a[1]) * m + p->wdl_a[2]) * m + p->wdl_a[3];
    if (!(a >= 1.0)) return fail(GN_E_INVALID, "win-rate model a(material %lld) = %g < 1", (long long)mc, a);
  }
  ctx->P = *p;
  ++ctx->graph_gen; // (the small-batch graphs hold the parameters they were captured with)
  return GN_OK;
}

int gn_net_info(const gn_ctx *ctx, int *big_l1, uint32_t *big_hash, int *small_l1, uint32_t *small_hash) {
  if (!ctx) return fail(GN_E_INVALID, "ctx is NULL");
  if (big_l1) *big_l1 = ctx->l1[BIG];
  if (big_hash) *big_hash = ctx->hash[BIG];
  if (small_l1) *small_l1 = ctx->l1[SMALL];
  if (small_hash) *small_hash = ctx->hash[SMALL];
  return GN_OK;
}

int gn_pack_fens(const char *const *fens, size_t n, gn_board *out, uint8_t *ok) {
  if (n && (!fens || !out)) return fail(GN_E_INVALID, "NULL argument");
  try {
    parallel_for(n, 4096, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        Board B;
        bool good = parse_fen(fens[i], B);
        if (good) pack(B, out[i]);
        else memset(&out[i], 0, sizeof(gn_board));
        if (ok) ok[i] = good;
      }
    });
  } catch (...) {
    return fail(GN_E_NOMEM, "thread start failed");
  }
  return GN_OK;
}

int gn_board_to_fen(const gn_board *board, char *buf, size_t buflen) {
  if (!board || !buf) return fail(GN_E_INVALID, "NULL argument");
  Board B;
  if (!unpack(*board, B)) return fail(GN_E_INVALID, "invalid board");
  if (board_to_fen(B, buf, buflen) < 0) return fail(GN_E_CAPACITY, "buffer too small");
  return GN_OK;
}

int gn_boards_to_fens(const gn_board *boards, size_t n, char *buf, size_t stride) {
  if (n && (!boards || !buf)) return fail(GN_E_INVALID, "NULL argument");
  if (stride < 100) return fail(GN_E_INVALID, "stride < 100");
  try {
    parallel_for(n, 4096, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        Board B;
        char *o = buf + i * stride;
        if (!unpack(boards[i], B) || board_to_fen(B, o, stride) < 0) o[0] = '\0';
      }
    });
  } catch (...) {
    return fail(GN_E_NOMEM, "thread start failed");
  }
  return GN_OK;
}

int gn_random_positions(uint64_t seed, size_t first_index, size_t n, int max_plies, gn_board *out) {
  if (n && !out) return fail(GN_E_INVALID, "NULL argument");
  if (max_plies < 0) return fail(GN_E_INVALID, "max_plies < 0");
  try {
    parallel_for(n, 256, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) pack(random_playout(seed + first_index + i, max_plies), out[i]);
    });
  } catch (...) {
    return fail(GN_E_NOMEM, "thread start failed");
  }
  return GN_OK;
}

int gn_evaluate_device(gn_ctx *ctx, int device_slot, const gn_board *d_boards, size_t n, int mode, gn_eval *d_out,
                       void *stream) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad context or device slot");
  if (n && (!d_boards || !d_out)) return fail(GN_E_INVALID, "NULL buffer");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  SeqGuard sg(*d, s);
  HIP_TRY(sg.e);
  int rc = evaluate_on(ctx, *d, d_boards, n, mode, d_out, s, nullptr);
  if (!rc) rc = resolve_scores(ctx, *d, d_boards, n, mode, d_out, nullptr, s);
  if (rc) return rc;
  HIP_TRY(sg.finish()); // blocking (gpu_nnue.h): d_out is written when the call returns
  return GN_OK;
}

int gn_time_evaluate_device(gn_ctx *ctx, int device_slot, const gn_board *d_boards, size_t n, int mode,
                            gn_eval *d_out, int iters, float *ms_total, float *per_kernel_ms, uint64_t *ft_rows) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad context or device slot");
  if (iters <= 0 || !ms_total) return fail(GN_E_INVALID, "bad iters / ms_total");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  SeqGuard sg(*d, d->stream);
  HIP_TRY(sg.e);
  std::vector<hipEvent_t> ev((size_t)iters * 5 + 2, nullptr);
  auto cleanup = [&] {
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
  };
  for (auto &e : ev)
    if (hipEventCreate(&e) != hipSuccess) {
      cleanup();
      return fail(GN_E_HIP, "hipEventCreate failed");
    }
  int rc = GN_OK;
  if (ft_rows) {
    HIP_TRY(d->sum.ensure(2));
    HIP_TRY(hipMemsetAsync(d->sum.p, 0, sizeof(unsigned long long), d->stream));
  }
  hipError_t he = hipEventRecord(ev[0], d->stream);
  for (int it = 0; it < iters && rc == GN_OK && he == hipSuccess; ++it) {
    rc = evaluate_on(ctx, *d, d_boards, n, mode, d_out, d->stream, per_kernel_ms ? &ev[2 + 5 * it] : nullptr,
                     ft_rows && it == 0 ? d->sum.p : nullptr);
    if (rc == GN_OK) rc = resolve_scores(ctx, *d, d_boards, n, mode, d_out, nullptr, d->stream);
  }
  if (rc == GN_OK && he == hipSuccess) he = hipEventRecord(ev[1], d->stream);
  if (rc == GN_OK && he == hipSuccess) he = hipEventSynchronize(ev[1]);
  if (rc == GN_OK && he == hipSuccess) he = hipEventElapsedTime(ms_total, ev[0], ev[1]);
  if (rc == GN_OK && he == hipSuccess && per_kernel_ms) {
    float acc[4] = {0, 0, 0, 0};
    for (int it = 0; it < iters && he == hipSuccess; ++it)
      for (int k = 0; k < 4 && he == hipSuccess; ++k) {
        float ms = 0;
        he = hipEventElapsedTime(&ms, ev[2 + 5 * it + k], ev[2 + 5 * it + k + 1]);
        acc[k] += ms;
      }
    for (int k = 0; k < 4; ++k) per_kernel_ms[k] = acc[k] / (float)iters;
  }
  cleanup();
  if (rc) return rc;
  if (ft_rows && he == hipSuccess) {
    unsigned long long r = 0;
    he = hipMemcpy(&r, d->sum.p, sizeof(r), hipMemcpyDeviceToHost);
    *ft_rows = r;
  }
  if (he != hipSuccess) return fail(GN_E_HIP, "timing failed: %s", hipGetErrorString(he));
  return GN_OK;
}

int gn_random_games_uci(uint64_t seed, size_t first_game, size_t n_games, int plies, char *buf, size_t stride) {
  if (n_games && !buf) return fail(GN_E_INVALID, "NULL argument");
  if (plies < 0 || plies > 1000) return fail(GN_E_INVALID, "plies out of range");
  if (stride < 6 * (size_t)plies + 1) return fail(GN_E_INVALID, "stride < 6 * plies + 1");
  try {
    parallel_for(n_games, 64, [&](size_t lo, size_t hi) {
      for (size_t g = lo; g < hi; ++g) {
        char *o = buf + g * stride;
        size_t len = 0;
        random_game(seed + first_game + g, plies, host_tables(), [&](int k, const Board &, uint16_t m) {
          if (!k || !m) return;
          if (len) o[len++] = ' ';
          len += (size_t)move_uci(m, o + len);
        });
        o[len] = '\0';
      }
    });
  } catch (...) {
    return fail(GN_E_NOMEM, "thread start failed");
  }
  return GN_OK;
}

int gn_random_positions_device(gn_ctx *ctx, int device_slot, uint64_t seed, size_t first_index, size_t n,
                               int max_plies, gn_board *d_out, void *stream) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad context or device slot");
  if (n && !d_out) return fail(GN_E_INVALID, "NULL buffer");
  if (max_plies < 0) return fail(GN_E_INVALID, "max_plies < 0");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  SeqGuard sg(*d, stream ? (hipStream_t)stream : d->stream);
  HIP_TRY(sg.e);
  HIP_TRY(launch_random_positions(seed, first_index, n, max_plies, d->tables, d_out, sg.s));
  return GN_OK;
}

int gn_device_alloc(gn_ctx *ctx, int device_slot, size_t bytes, void **ptr) {
  Dev *d = slot(ctx, device_slot);
  if (!d || !ptr) return fail(GN_E_INVALID, "bad argument");
  HIP_TRY(hipSetDevice(d->id));
  if (hipMalloc(ptr, std::max<size_t>(bytes, 1)) != hipSuccess) return fail(GN_E_NOMEM, "hipMalloc(%zu) failed", bytes);
  return GN_OK;
}

int gn_device_free(gn_ctx *ctx, int device_slot, void *ptr) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad argument");
  HIP_TRY(hipSetDevice(d->id));
  if (ptr) HIP_TRY(hipFree(ptr));
  return GN_OK;
}

int gn_memcpy_h2d(gn_ctx *ctx, int device_slot, void *dst, const void *src, size_t bytes) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  SeqGuard sg(*d, d->stream);
  HIP_TRY(sg.e);
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return GN_OK;
}

int gn_memcpy_d2h(gn_ctx *ctx, int device_slot, void *dst, const void *src, size_t bytes) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  SeqGuard sg(*d, d->stream);
  HIP_TRY(sg.e);
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return GN_OK;
}

int gn_synchronize(gn_ctx *ctx, int device_slot) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  if (d->done_on) HIP_TRY(hipEventSynchronize(d->done)); // the last launch sequence, on whatever stream
  HIP_TRY(hipStreamSynchronize(d->stream));
  return GN_OK;
}

int gn_evaluate_batch_mode(gn_ctx *ctx, const char *const *fens, size_t n, int mode, gn_eval *out) {
  if (!ctx) return fail(GN_E_INVALID, "ctx is NULL");
  if (n && (!fens || !out)) return fail(GN_E_INVALID, "NULL argument");
  if (!n) return GN_OK;
  try {
    std::vector<gn_board> boards(n);
    int rc = gn_pack_fens(fens, n, boards.data(), nullptr);
    if (rc) return rc;
    return evaluate_coalesced(ctx, boards.data(), n, mode, out);
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

int gn_evaluate_batch(gn_ctx *ctx, const char *const *fens, size_t n, gn_eval *out) {
  return gn_evaluate_batch_mode(ctx, fens, n, GN_MODE_FULL, out);
}

int gn_expand_device(gn_ctx *ctx, int device_slot, const gn_board *d_parents, size_t n, int mode,
                     gn_eval *d_parent_out, uint32_t *d_offsets, gn_board *d_children, uint16_t *d_moves,
                     gn_eval *d_child_out, size_t cap, size_t *total, void *stream) {
  Dev *d = slot(ctx, device_slot);
  if (!d || !total) return fail(GN_E_INVALID, "bad argument");
  if (n && (!d_parents || !d_offsets)) return fail(GN_E_INVALID, "NULL buffer");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  SeqGuard sg(*d, s);
  HIP_TRY(sg.e);
  *total = 0;
  if (!n) return GN_OK;
  if (!d_children || !d_moves || !d_child_out) return fail(GN_E_INVALID, "NULL child buffer");
  size_t t = 0;
  int rc = generate_children(*d, d_parents, n, d_children, cap, d_moves, ctx->incremental, &t, s, nullptr, nullptr,
                             chain_len(ctx, *d, n), plan_path(ctx, *d, mode), mode == GN_MODE_BIG);
  *total = t;
  if (t > 0xFFFFFFFFull) return fail(GN_E_CAPACITY, "%zu children exceed 32-bit offsets", t);
  HIP_TRY(launch_offsets_u32(d->offsets.p, n + 1, d_offsets, s));
  if (rc) {
    HIP_TRY(hipStreamSynchronize(s));
    return rc;
  }
  rc = expand_evaluate(ctx, *d, d_parents, n, d_children, t, mode, d_parent_out, d_child_out, s, nullptr);
  const Replies rp{d_child_out, d_moves}; // the replies this expansion evaluated
  if (!rc) rc = resolve_scores(ctx, *d, d_parents, n, mode, d_parent_out, nullptr, s, 2, &rp);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return check_plan(*d, s);
}

// Depth 2: the children of gn_expand_device's children.  Level 2 is
// the same machinery with the children as parents: they arrive in sibling order, so a
// block of consecutive siblings refreshes each from its predecessor's king-cache row
// (plan_kernel: cache row + the placement difference, a few rows instead of ~30) and
// every grandchild is incremental from its parent's accumulator.  The children are
// evaluated again at level 2 (as parents); those results must equal level 1's and are
// compared on the device (GN_E_HIP if not: an internal consistency check).
int gn_expand2_device(gn_ctx *ctx, int device_slot, const gn_board *d_parents, size_t n, int mode,
                      gn_eval *d_parent_out, uint32_t *d_offsets, gn_board *d_children, uint16_t *d_moves,
                      gn_eval *d_child_out, size_t cap, uint32_t *d_goffsets, uint16_t *d_gmoves,
                      gn_eval *d_grand_out, size_t gcap, size_t *total, size_t *gtotal, void *stream) {
  Dev *d = slot(ctx, device_slot);
  if (!d || !total || !gtotal) return fail(GN_E_INVALID, "bad argument");
  if (n && (!d_parents || !d_offsets)) return fail(GN_E_INVALID, "NULL buffer");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  SeqGuard sg(*d, s);
  HIP_TRY(sg.e);
  *total = *gtotal = 0;
  if (!n) return GN_OK;
  // a size query (NULL child buffers or too small): the counts, GN_E_CAPACITY
  size_t t = 0;
  if (!d_children || !d_moves || !d_child_out || !cap) {
    HIP_TRY(count_children(*d, d_parents, n, s, &t));
    *total = t;
    return t ? fail(GN_E_CAPACITY, "%zu children exceed capacity %zu", t, cap) : GN_OK;
  }
  // level 1
  int rc = generate_children(*d, d_parents, n, d_children, cap, d_moves, ctx->incremental, &t, s, nullptr, nullptr,
                             chain_len(ctx, *d, n), plan_path(ctx, *d, mode), mode == GN_MODE_BIG);
  *total = t;
  if (t > 0xFFFFFFFFull) return fail(GN_E_CAPACITY, "%zu children exceed 32-bit offsets", t);
  HIP_TRY(launch_offsets_u32(d->offsets.p, n + 1, d_offsets, s));
  if (rc) {
    HIP_TRY(hipStreamSynchronize(s));
    return rc;
  }
  rc = expand_evaluate(ctx, *d, d_parents, n, d_children, t, mode, d_parent_out, d_child_out, s, nullptr);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  if ((rc = check_plan(*d, s)) != GN_OK) return rc;
  const Replies rp{d_child_out, d_moves}; // level 1's replies
  if ((rc = resolve_scores(ctx, *d, d_parents, n, mode, d_parent_out, nullptr, s, 2, &rp)) != GN_OK) return rc;
  if (!t) {
    HIP_TRY(hipMemsetAsync(d_goffsets, 0, sizeof(uint32_t), s));
    HIP_TRY(hipStreamSynchronize(s));
    return GN_OK;
  }
  // level 2: the children as parents (their grandchildren boards stay library-internal)
  size_t g = 0;
  if (!d_goffsets || !d_gmoves || !d_grand_out || !gcap) {
    HIP_TRY(count_children(*d, d_children, t, s, &g));
    *gtotal = g;
    return g ? fail(GN_E_CAPACITY, "%zu grandchildren exceed capacity %zu", g, gcap) : GN_OK;
  }
  rc = generate_children(*d, d_children, t, nullptr, gcap, d_gmoves, ctx->incremental, &g, s, nullptr, nullptr,
                         chain_len(ctx, *d, t), plan_path(ctx, *d, mode), mode == GN_MODE_BIG);
  *gtotal = g;
  if (g > 0xFFFFFFFFull) return fail(GN_E_CAPACITY, "%zu grandchildren exceed 32-bit offsets", g);
  HIP_TRY(launch_offsets_u32(d->offsets.p, t + 1, d_goffsets, s));
  if (rc) {
    HIP_TRY(hipStreamSynchronize(s));
    return rc;
  }
  HIP_TRY(d->io_out.ensure(t));
  // (the children as parents are child records here too: compared with level 1's below)
  rc = expand_evaluate(ctx, *d, d_children, t, d->frontier[1].p, g, mode, d->io_out.p, d_grand_out, s, nullptr,
                       nullptr, false);
  if (rc) return rc;
  // the children evaluated twice (level 1 as children, level 2 as parents) must agree
  HIP_TRY(d->sum.ensure(2));
  HIP_TRY(hipMemsetAsync(d->sum.p, 0, 2 * sizeof(unsigned long long), s));
  HIP_TRY(launch_checksum(d_child_out, t * sizeof(gn_eval), d->sum.p, s));
  HIP_TRY(launch_checksum(d->io_out.p, t * sizeof(gn_eval), d->sum.p + 1, s));
  unsigned long long cs[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(cs, d->sum.p, sizeof(cs), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if ((rc = check_plan(*d, s)) != GN_OK) return rc;
  if (cs[0] != cs[1]) return fail(GN_E_HIP, "depth 2: the children's level-1 and level-2 evaluations differ");
  return GN_OK;
}

int gn_time_expand_device(gn_ctx *ctx, int device_slot, const gn_board *d_parents, size_t n, int mode, int iters,
                          float *ms_total, size_t *total, float *stage_ms, uint64_t *ft_rows, gn_eval *d_parent_out,
                          uint32_t *d_offsets, uint16_t *d_moves, gn_eval *d_child_out, size_t cap) {
  Dev *d = slot(ctx, device_slot);
  if (!d || !ms_total || !total || iters <= 0) return fail(GN_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  hipStream_t s = d->stream;
  SeqGuard sg(*d, s);
  HIP_TRY(sg.e);
  // start, [count+scan], [total read], [write], [classify], [small], [big], [finalize], the
  // planned big net's plan -> stream boundary, [score rule] (ends at e[9]), and the stream ->
  // finish boundary (e[10])
  const int NE = 12;
  std::vector<hipEvent_t> ev((size_t)iters * NE + 2, nullptr);
  auto cleanup = [&] {
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
  };
  for (auto &e : ev)
    if (hipEventCreate(&e) != hipSuccess) {
      cleanup();
      return fail(GN_E_HIP, "hipEventCreate failed");
    }
  int rc = GN_OK;
  size_t t = 0;
  HIP_TRY(d->sum.ensure(2)); // [0] rows by write_children's formula, [1] rows the row stream gathered
  HIP_TRY(hipMemsetAsync(d->sum.p, 0, 2 * sizeof(unsigned long long), s));
  hipError_t he = hipEventRecord(ev[0], s);
  // the expansion pipeline (GN_OPT_EXPAND_PIPELINE): expansion it + 1's front half (children,
  // plan) on the device's second stream, into the other buffer set, while expansion it's finalize
  // and score rule run; its row stream waits for that plan
  const bool pipe = ctx->pipeline && plan_path(ctx, *d, mode) && ctx->incremental && iters > 1;
  if (pipe && he == hipSuccess) {
    hipStream_t B = d->front;
    size_t tn = 0; // the children of the expansion whose front ran last
    auto front = [&](int it) -> int {
      hipEvent_t *e = &ev[2 + (size_t)NE * it];
      HIP_TRY(hipEventRecord(e[0], B));
      // (moves into the set's own buffer: the caller's is written once, after the last expansion)
      int r = generate_children(*d, d_parents, n, nullptr, cap, nullptr, true, &tn, B, e + 1, nullptr,
                                chain_len(ctx, *d, n), true, mode == GN_MODE_BIG);
      if (r) return r;
      if (d_child_out && tn > cap) return fail(GN_E_CAPACITY, "%zu children exceed capacity %zu", tn, cap);
      r = expand_evaluate(ctx, *d, d_parents, n, d->frontier[1].p, tn, mode, nullptr, nullptr, B, e + 4,
                          it == 0 ? d->sum.p + 1 : nullptr, true, EXP_FRONT);
      if (r) return r;
      HIP_TRY(hipEventRecord(d->ev_planned, B));
      return GN_OK;
    };
    // the front starts after what the stream holds so far (the sequence guard's wait, the reset)
    he = hipEventRecord(d->ev_streamed, s);
    if (he == hipSuccess) he = hipStreamWaitEvent(B, d->ev_streamed, 0);
    if (he == hipSuccess) rc = front(0);
    t = tn;
    d->part_locked = true; // (front(0) sized the partial sums; later fronts run beside a back half)
    struct Unlock {
      Dev &d;
      ~Unlock() { d.part_locked = false; }
    } unlock{*d};
    HIP_TRY(d->io_out.ensure(n));
    HIP_TRY(d->io_out2.ensure(std::max<size_t>(t, 1)));
    gn_eval *po = d_parent_out ? d_parent_out : d->io_out.p, *co = d_child_out ? d_child_out : d->io_out2.p;
    for (int it = 0; it < iters && rc == GN_OK && he == hipSuccess; ++it) {
      hipEvent_t *e = &ev[2 + (size_t)NE * it];
      if ((he = hipStreamWaitEvent(s, d->ev_planned, 0)) != hipSuccess) break;
      rc = expand_evaluate(ctx, *d, d_parents, n, d->frontier[1].p, t, mode, po, co, s, e + 4, nullptr, true,
                           EXP_BACK);
      if (rc) break;
      const bool more = it + 1 < iters;
      if (more) { // the next front, after this row stream (it overwrites the plan's lists)
        swap_sets(*d);
        he = ctx->pipeline == 2 ? hipSuccess : hipStreamWaitEvent(B, e[10], 0);
        if (he == hipSuccess) rc = front(it + 1);
        swap_sets(*d);
        if (rc || he != hipSuccess) break;
      }
      const Replies rp{co, d->child_moves};
      rc = resolve_scores(ctx, *d, d_parents, n, mode, po, nullptr, s, 2, &rp);
      if (rc == GN_OK) he = hipEventRecord(e[9], s);
      if (more) swap_sets(*d), t = tn;
    }
    if (rc == GN_OK && he == hipSuccess && d_moves && t)
      he = hipMemcpyAsync(d_moves, d->child_moves, t * sizeof(uint16_t), hipMemcpyDeviceToDevice, s);
  }
  for (int it = 0; !pipe && it < iters && rc == GN_OK && he == hipSuccess; ++it) {
    hipEvent_t *e = &ev[2 + (size_t)NE * it];
    he = hipEventRecord(e[0], s);
    if (he != hipSuccess) break;
    // rows by write_children's formula only when no planned row stream counts them (a
    // per-wave atomic over every child would sit in the timed region)
    const bool planned = plan_path(ctx, *d, mode);
    rc = generate_children(*d, d_parents, n, nullptr, cap, d_moves, ctx->incremental, &t, s, e + 1,
                           it == 0 && !planned ? d->sum.p : nullptr, chain_len(ctx, *d, n), planned,
                           mode == GN_MODE_BIG);
    if (rc) break;
    if (d_child_out && t > cap) {
      rc = fail(GN_E_CAPACITY, "%zu children exceed capacity %zu", t, cap);
      break;
    }
    HIP_TRY(d->io_out.ensure(n));
    HIP_TRY(d->io_out2.ensure(std::max<size_t>(t, 1)));
    gn_eval *po = d_parent_out ? d_parent_out : d->io_out.p;
    rc = expand_evaluate(ctx, *d, d_parents, n, d->frontier[1].p, t, mode, po,
                         d_child_out ? d_child_out : d->io_out2.p, s, e + 4, it == 0 ? d->sum.p + 1 : nullptr);
    const Replies rp{d_child_out ? d_child_out : d->io_out2.p, d->child_moves}; // this expansion's replies
    if (rc == GN_OK) rc = resolve_scores(ctx, *d, d_parents, n, mode, po, nullptr, s, 2, &rp);
    if (rc == GN_OK) he = hipEventRecord(e[9], s);
  }
  if (rc == GN_OK && he == hipSuccess && d_offsets) he = launch_offsets_u32(d->offsets.p, n + 1, d_offsets, s);
  if (rc == GN_OK && he == hipSuccess) he = hipEventRecord(ev[1], s);
  if (rc == GN_OK && he == hipSuccess) he = hipEventSynchronize(ev[1]);
  if (rc == GN_OK && he == hipSuccess) he = hipEventElapsedTime(ms_total, ev[0], ev[1]);
  // stage k from event k to k + 1 (score: 7 -> 9).  Pipelined, the front's stages are on the second
  // stream and the big net is the plan (5 -> 8) plus the stream (11 -> 10, after its wait)
  if (rc == GN_OK && he == hipSuccess && stage_ms) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int it = 0; it < iters && he == hipSuccess; ++it)
      for (int k = 0; k < 8 && he == hipSuccess; ++k) {
        float ms = 0, ms2 = 0;
        const size_t o = 2 + (size_t)NE * it;
        if (pipe && k == 5) {
          he = hipEventElapsedTime(&ms, ev[o + 5], ev[o + 8]);
          if (he == hipSuccess) he = hipEventElapsedTime(&ms2, ev[o + 11], ev[o + 6]);
        } else {
          he = hipEventElapsedTime(&ms, ev[o + k], ev[o + (k < 7 ? k + 1 : 9)]);
        }
        acc[k] += ms + ms2;
      }
    for (int k = 0; k < 8; ++k) stage_ms[k] = acc[k] / (float)iters;
  }
  if (rc == GN_OK && he == hipSuccess && d->planned) { // the big net's two kernels apart
    float pl = 0, st = 0, fi = 0;
    for (int it = 0; it < iters && he == hipSuccess; ++it) {
      float a = 0, b = 0, c = 0;
      const size_t o = 2 + (size_t)NE * it;
      he = hipEventElapsedTime(&a, ev[o + 5], ev[o + 8]);
      if (he == hipSuccess) he = hipEventElapsedTime(&b, ev[o + (pipe ? 11 : 8)], ev[o + 10]); // the stream launches
      if (he == hipSuccess) he = hipEventElapsedTime(&c, ev[o + 10], ev[o + 6]);  // the sliced stream's finish
      pl += a, st += b, fi += c;
    }
    d->plan_ms = pl / (float)iters, d->stream_ms = st / (float)iters, d->finish_ms = fi / (float)iters;
  }
  cleanup();
  *total = t;
  if (rc) return rc;
  if (he == hipSuccess && (rc = check_plan(*d, s)) != GN_OK) return rc;
  if (he == hipSuccess && pipe) { // (the other set's expansion too)
    swap_sets(*d);
    rc = check_plan(*d, s);
    swap_sets(*d);
    if (rc) return rc;
  }
  if (ft_rows && he == hipSuccess) {
    unsigned long long r[2] = {0, 0};
    he = hipMemcpy(r, d->sum.p, sizeof(r), hipMemcpyDeviceToHost);
    *ft_rows = ctx->incremental ? (r[1] ? r[1] : r[0]) : 0; // the row stream's own count when it ran
  }
  if (he != hipSuccess) return fail(GN_E_HIP, "timing failed: %s", hipGetErrorString(he));
  return GN_OK;
}

int gn_checksum_device(gn_ctx *ctx, int device_slot, const void *d_ptr, size_t bytes, uint64_t *sum) {
  Dev *d = slot(ctx, device_slot);
  if (!d || !sum || (bytes && !d_ptr)) return fail(GN_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  SeqGuard sg(*d, d->stream);
  HIP_TRY(sg.e);
  HIP_TRY(d->sum.ensure(2));
  HIP_TRY(hipMemsetAsync(d->sum.p, 0, sizeof(unsigned long long), d->stream));
  HIP_TRY(launch_checksum(d_ptr, bytes, d->sum.p, d->stream));
  unsigned long long r = 0;
  HIP_TRY(hipMemcpyAsync(&r, d->sum.p, sizeof(r), hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  *sum = r;
  return GN_OK;
}

int gn_random_games_device(gn_ctx *ctx, int device_slot, uint64_t seed, size_t first_game, size_t n_games, int plies,
                           gn_board *d_out, void *stream) {
  Dev *d = slot(ctx, device_slot);
  if (!d) return fail(GN_E_INVALID, "bad context or device slot");
  if (n_games && !d_out) return fail(GN_E_INVALID, "NULL buffer");
  if (plies < 0 || plies > 1000) return fail(GN_E_INVALID, "plies out of range");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  SeqGuard sg(*d, stream ? (hipStream_t)stream : d->stream);
  HIP_TRY(sg.e);
  HIP_TRY(launch_random_games(seed, first_game, n_games, plies, d->tables, d_out, sg.s));
  return GN_OK;
}

int gn_set_option(gn_ctx *ctx, int option, int64_t value) {
  if (!ctx) return fail(GN_E_INVALID, "ctx is NULL");
  ++ctx->graph_gen; // (the small-batch graphs hold the options they were captured with)
  switch (option) {
  case GN_OPT_INCREMENTAL_CHILDREN:
    ctx->incremental = value != 0;
    return GN_OK;
  case GN_OPT_XCD_SWIZZLE:
    ctx->swizzle = (int)(value & 15);
    return GN_OK;
  case GN_OPT_KING_SORT:
    if (value < 0 || value > 2) return fail(GN_E_INVALID, "king sort must be 0, 1 or 2");
    ctx->king_sort = (int)value;
    return GN_OK;
  case GN_OPT_KING_CACHE:
    ctx->king_cache = value != 0;
    return GN_OK;
  case GN_OPT_CHAIN:
    if (value < -(1 << 20) || value > (1 << 20)) return fail(GN_E_INVALID, "chain length out of range");
    ctx->chain = (int)value;
    return GN_OK;
  case GN_OPT_STREAM_SLICES:
    if (value != 1 && value != 3) return fail(GN_E_INVALID, "stream slices must be 1 or 3");
    ctx->stream_slices = (int)value;
    return GN_OK;
  case GN_OPT_CHUNK_PARENTS:
    if (value < 0) return fail(GN_E_INVALID, "chunk size < 0");
    ctx->chunk_parents = value;
    return GN_OK;
  case GN_OPT_COALESCE:
    ctx->coalesce = value != 0;
    return GN_OK;
  case GN_OPT_FAST_BATCH:
    ctx->fast_batch = value != 0;
    return GN_OK;
  case GN_OPT_EXPAND_PIPELINE:
    if (value < 0 || value > 2) return fail(GN_E_INVALID, "GN_OPT_EXPAND_PIPELINE %lld not in 0..2", (long long)value);
    ctx->pipeline = (int)value;
    return GN_OK;
  default:
    return fail(GN_E_INVALID, "unknown option %d", option);
  }
}

int gn_get_option(const gn_ctx *ctx, int option, int64_t *value) {
  if (!ctx || !value) return fail(GN_E_INVALID, "NULL argument");
  switch (option) {
  case GN_OPT_INCREMENTAL_CHILDREN:
    *value = ctx->incremental;
    return GN_OK;
  case GN_OPT_XCD_SWIZZLE:
    *value = ctx->swizzle;
    return GN_OK;
  case GN_OPT_KING_SORT:
    *value = ctx->king_sort;
    return GN_OK;
  case GN_OPT_KING_CACHE:
    *value = ctx->king_cache;
    return GN_OK;
  case GN_OPT_CHAIN:
    *value = ctx->chain;
    return GN_OK;
  case GN_OPT_STREAM_SLICES:
    *value = ctx->stream_slices;
    return GN_OK;
  case GN_OPT_CHUNK_PARENTS:
    *value = ctx->chunk_parents;
    return GN_OK;
  case GN_OPT_COALESCE:
    *value = ctx->coalesce;
    return GN_OK;
  case GN_OPT_FAST_BATCH:
    *value = ctx->fast_batch;
    return GN_OK;
  case GN_OPT_EXPAND_PIPELINE:
    *value = ctx->pipeline;
    return GN_OK;
  case GN_STAT_FAST_BATCHES:
    *value = (int64_t)ctx->fast_runs.load();
    return GN_OK;
  case GN_STAT_FAST_FALLBACKS:
    *value = (int64_t)ctx->fast_fallbacks.load();
    return GN_OK;
  case GN_STAT_BATCH_LAUNCHES:
  case GN_STAT_BATCH_CALLS: { // cumulative since load (the coalescer's counters)
    auto &C = const_cast<gn_ctx *>(ctx)->co;
    std::lock_guard<std::mutex> lk(C.mu);
    *value = (int64_t)(option == GN_STAT_BATCH_LAUNCHES ? C.launches : C.calls);
    return GN_OK;
  }
  case GN_STAT_PLAN_NS:
  case GN_STAT_STREAM_NS:
  case GN_STAT_FINISH_NS: { // read-only: the last gn_time_expand_device's planned kernels (max over devices)
    float m = 0;
    for (auto &dp : ctx->devs)
      m = std::max(m, option == GN_STAT_PLAN_NS     ? dp->plan_ms
                      : option == GN_STAT_STREAM_NS ? dp->stream_ms
                                                    : dp->finish_ms);
    *value = (int64_t)((double)m * 1e6);
    return GN_OK;
  }
  case GN_STAT_HOST_PARSE_NS:
  case GN_STAT_HOST_TOTAL_NS:
    *value = (int64_t)((option == GN_STAT_HOST_PARSE_NS ? ctx->t_parse : ctx->t_total) * 1e6);
    return GN_OK;
  case GN_STAT_HOST_UPLOAD_NS:
  case GN_STAT_HOST_REPLAY_NS:
  case GN_STAT_HOST_COMPUTE_NS:
  case GN_STAT_HOST_DOWNLOAD_NS:
  case GN_STAT_HOST_TAIL_NS: { // the last host-buffer call, max over devices
    double m = 0;
    for (auto &dp : ctx->devs) {
      const Dev &d = *dp;
      m = std::max(m, option == GN_STAT_HOST_UPLOAD_NS    ? d.t_upload
                      : option == GN_STAT_HOST_REPLAY_NS  ? d.t_replay
                      : option == GN_STAT_HOST_COMPUTE_NS ? d.t_compute
                      : option == GN_STAT_HOST_DOWNLOAD_NS ? d.t_download
                                                           : d.t_tail);
    }
    *value = (int64_t)(m * 1e6);
    return GN_OK;
  }
  case GN_STAT_SCRATCH_PADS: { // read-only: the last planned expansion's GN_SCR_GAP no-op entries, summed
    int64_t sum = 0;
    for (auto &dp : ctx->devs) {
      Dev &d = *dp;
      std::lock_guard<std::mutex> lk(d.mu);
      if (!d.pstat.p) continue;
      HIP_TRY(hipSetDevice(d.id));
      if (d.done_on) HIP_TRY(hipEventSynchronize(d.done));
      unsigned long long v = 0;
      HIP_TRY(hipMemcpy(&v, d.pstat.p, sizeof(v), hipMemcpyDeviceToHost));
      sum += (int64_t)v;
    }
    *value = sum;
    return GN_OK;
  }
  default:
    return fail(GN_E_INVALID, "unknown option %d", option);
  }
}

int gn_expand_and_evaluate(gn_ctx *ctx, const char *const *parent_fens, size_t n, int mode, gn_eval *parent_out,
                           uint32_t *child_offsets, uint16_t *child_moves, gn_child *child_out, size_t cap) {
  if (!slot(ctx, 0)) return fail(GN_E_INVALID, "bad context");
  if (n && (!parent_fens || !child_offsets)) return fail(GN_E_INVALID, "NULL argument");
  if (!n) {
    if (child_offsets) child_offsets[0] = 0;
    return GN_OK;
  }
  try {
    const auto T0 = Clock::now();
    reset_host_stats(ctx);
    std::vector<gn_board> boards(n);
    int rc = gn_pack_fens(parent_fens, n, boards.data(), nullptr);
    if (rc) return rc;
    ctx->t_parse = ms_since(T0);
    rc = expand_boards_host(ctx, boards.data(), n, mode, parent_out, child_offsets, child_moves, child_out, cap);
    ctx->t_total = ms_since(T0);
    return rc;
  } catch (const std::bad_alloc &) {
    return fail(GN_E_NOMEM, "host allocation failed");
  } catch (...) {
    return fail(GN_E_INVALID, "unexpected exception");
  }
}

int gn_perft(gn_ctx *ctx, const char *fen, int depth, uint64_t *nodes) {
  Dev *d = slot(ctx, 0);
  if (!d || !fen || !nodes) return fail(GN_E_INVALID, "bad argument");
  Board B;
  if (!parse_fen(fen, B)) return fail(GN_E_INVALID, "bad FEN");
  if (depth <= 0) {
    *nodes = 1;
    return GN_OK;
  }
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  hipStream_t s = d->stream;
  SeqGuard sg(*d, s);
  HIP_TRY(sg.e);
  gn_board root;
  pack(B, root);
  HIP_TRY(d->frontier[0].ensure(1));
  HIP_TRY(hipMemcpyAsync(d->frontier[0].p, &root, sizeof(root), hipMemcpyHostToDevice, s));
  size_t n = 1;
  for (int level = 1; level < depth; ++level) {
    size_t total = 0;
    int rc = generate_children(*d, d->frontier[0].p, n, nullptr, 0, nullptr, false, &total, s, nullptr);
    if (rc) return rc;
    std::swap(d->frontier[0], d->frontier[1]);
    n = total;
    if (!n) break;
  }
  unsigned long long sum = 0;
  if (n) {
    HIP_TRY(d->sum.ensure(1));
    HIP_TRY(hipMemsetAsync(d->sum.p, 0, sizeof(unsigned long long), s));
    HIP_TRY(launch_count_sum(d->frontier[0].p, n, d->tables, d->sum.p, s));
    HIP_TRY(hipMemcpyAsync(&sum, d->sum.p, sizeof(sum), hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  *nodes = sum;
  return GN_OK;
}

} // extern "C"
