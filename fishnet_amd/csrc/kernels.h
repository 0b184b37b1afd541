// kernels.h — host-side launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "nnue.h"

// Row-ring depth of the planned expansion's stream (stream.hip: entries in flight per wave,
// 4 or 8), and GN_SCR_GAP, the least distance in entries of one list from a king-cache store to
// a later load of that row (the plan pads the lists to keep it and asserts it: error bit 2).
// The ring issues an entry's row loads while consuming the entry GN_RING before it, and the
// store happens while consuming its own entry, so at a distance >= GN_RING the load is issued
// after the store, by the same lanes, to the same address.  One work-item's later load of an
// address it stored needs no wait on this hardware: hipcc itself emits `global_store_dword`
// directly followed by `global_load_dword` for C++ `p[i] = x; y = p[i ^ j];`
// (tests/test_host.py::test_same_address_store_then_load_needs_no_wait compiles exactly that
// and checks), i.e. one wave's vector-memory operations reach one address in issue order.
// -DGN_SCR_GAP=7 (2 * GN_RING - 1) is the stricter variant: the ring's vmcnt(2 * GN_RING - 2)
// waits then retire the store before the load issues (vmcnt counts loads and stores together
// in issue order, MI355X_MICROARCH.md "s_waitcnt vmcnt(N)"); measured 2.9 % slower stream.
#ifndef GN_RING
#define GN_RING 4
#endif
// the column-sliced stream's ring (stream_eval_kernel<3072, 3>): 4, 5 or 6 entries per wave
#ifndef GN_SLICE_RING
#define GN_SLICE_RING 4
#endif
#ifndef GN_SCR_GAP // (the plan serves both streams: the deeper ring's distance)
#define GN_SCR_GAP (GN_RING > GN_SLICE_RING ? GN_RING : GN_SLICE_RING)
#endif
// Workgroup size of the expansion's front kernels (count_children, child_moves, child_boards,
// block_keys, plan_kernel).  The expansion pipeline runs them beside the row stream, whose
// 2-wave workgroups hold every wave slot of a CU: a front workgroup is dispatched only where
// enough stream workgroups have ended at once.  2 waves (128): per step 150.8 against 151.9 ms
// with 4 (256) and 153.0 with 1 (64), which runs the front fully beside the stream and slows
// the stream by as much (round 6, profiles/r06/ab_r06p_front_wg.log).
#ifndef GN_FRONT_WG
#define GN_FRONT_WG 128
#endif
static_assert(GN_FRONT_WG == 64 || GN_FRONT_WG == 128 || GN_FRONT_WG == 256, "front workgroups of 1, 2 or 4 waves");

// Spare entries at the end of each block's entry region (plan_kernel, stream_eval_kernel): the
// stream's scalar prefetch of the entries two ring revolutions ahead reads up to 2 * ring + 8 - 1
// entries past its position, so a list ending at the region less the spares never reads past it.
constexpr unsigned ENT_SPARE = 32;

// The column-sliced stream's fc_0 partial sums: one array per slice (default), which
// slice_finish_kernel adds; or, with -DGN_PART_INPLACE (A/B only), one array that each slice
// s > 0 adds its sums to in place, reading slice s - 1's at the tile's start.  In place measured
// slower (round 5: finish 5.44 -> 2.75 ms, but each later stream launch +2.1 ms: the prefetch
// misses to HBM and, vector-memory completion being in order, holds up the ring's next loads).
// GN_PART_SLICES: the arrays launch_plan_stream's part holds.
#ifdef GN_PART_INPLACE
#define GN_PART_SLICES 1
#else
#define GN_PART_SLICES 3
#endif

namespace gn {

// NetworkOutput {psqt / 16, positional / 16} for every position whose
// need[i] != 0 (need == nullptr: all); other entries of out are untouched.
// perm (optional): slot q evaluates boards[perm[q]] and writes out[perm[q]].
// swz: XCD-aware tile order (each XCD gets a contiguous range of tiles).
// rows_out (optional): += FT rows the gather reads (common-row base counted once per tile).
// cls (the small net, mode FULL): the kernel selects the positions itself (classify_kernel's rule:
// need_small / need_big written for every position, need ignored) and applies reeval_kernel's rule to
// the small net's outputs (need_big set where |nnue| < reeval_threshold): one launch for three.
hipError_t launch_eval_net(const NetDevice &net, const gn_board *boards, const uint8_t *need, size_t n,
                           int2 *out, const uint32_t *perm, int swz, hipStream_t s,
                           unsigned long long *rows_out = nullptr, const gn_eval_params *cls = nullptr,
                           uint8_t *need_small = nullptr, uint8_t *need_big = nullptr);
// *out += position-sensitive checksum of bytes at p (caller zeroes *out)
hipError_t launch_checksum(const void *p, size_t bytes, unsigned long long *out, hipStream_t s);
// permutation of [0, n) ordering positions by (white king, black king) square, then
// (placement) by 30 home-square bits, one per square of ranks 1, 2, 7, 8 without
// e1 / e8, set when the start position's piece still stands there
// (king_keys_kernel), which serve the big net's common-row base; kings only
// (16-bit keys) otherwise
// order[]: the nblk blocks (K consecutive parents each) sorted by their middle parent's
// king squares (stream_eval_kernel's XCD-local order); keys / idx / keys_out: nblk scratch.
hipError_t block_order(const gn_board *parents, size_t n, uint32_t K, uint32_t nblk, uint16_t *keys, uint32_t *idx,
                       uint16_t *keys_out, uint32_t *order, void *&temp, size_t &temp_bytes, hipStream_t s);
hipError_t king_sort(const gn_board *boards, size_t n, uint64_t *keys, uint32_t *idx, uint64_t *keys_out,
                     uint32_t *perm, bool placement, void *&temp, size_t &temp_bytes, hipStream_t s);
// Incremental evaluation of parents + all their children with the small net (L1 = 128;
// expand_eval_kernel, one workgroup per parent; children of parent p are
// [offsets[p], offsets[p+1]) with deltas[]); need_* select what this net evaluates
// (nullptr: all).  The big nets always run planned (launch_plan_stream).
hipError_t launch_expand_net(const NetDevice &net, const gn_board *parents, size_t n, const uint64_t *offsets,
                             const gn_board *children, const ChildDelta *deltas, const uint8_t *need_parent,
                             const uint8_t *need_child, int2 *out_parent, int2 *out_child, int swz, hipStream_t s);
// Planned expansion (stream.hip): one descriptor per tile of <= 16 consecutive slots of a
// block (slots = [parent, its children, next parent, ...] of the block's consecutive
// parents) with <= 2 buckets among its evaluated slots.  e_end: list 0 / list 1 entries
// of the block up to the end of this tile (padded to a multiple of 4); p_first: the
// parent owning slot 0; first: the block-relative index of slot 0; meta[t]: bit 0
// evaluated, bits 1-3 bucket, bit 4 a parent slot, bit 5 the slot's side to move;
// psq[t][side]: the slot's PSQT accumulators at its bucket (side 0: the perspective to move).
struct TileDesc {
  uint32_t e_end[2];
  uint32_t p_first;
  uint32_t first;
  uint8_t meta[16];
  int32_t psq[16][2];
  int16_t adj[16]; // a child slot's output index minus its position (the chained walk's reorder)
};
static_assert(sizeof(TileDesc) == 192, "TileDesc is 192 bytes");
// Tiles of a block start at tiles + (pbeg + offsets[pbeg]) / 16 + (K + 2) * block (btiles[block]
// of them), entries at ent + eoff[pbeg] + 16 * block (list 0 upward, list 1 downward from
// the region's end, eoff = exclusive scan of write_children's per-parent entry bounds).
// One call plans and evaluates blocks [b0, b1) of the n parents (every index absolute, so
// block ranges can run as a pipeline on different streams).  pool: 88 words (scratch-slot
// bits, then 8 block claim counters per stream launch), zeroed by the caller before each call; err: bit 0 entry overflow, bit 1 no scratch slot, bit 2 a
// king-cache load closer than GN_SCR_GAP entries to its list's last store to scratch.
// rows_out: += FT rows the stream gathers (bias, carry and king-cache rows included);
// pads_out (optional): += no-op entries the plan inserted to keep GN_SCR_GAP.
// order: block order of the stream (block_order) or NULL; mid: recorded between the kernels.
// slices == 3 (L1 3072; part, pinfo non-null): the stream runs as three launches over 1,024
// columns each (stream_eval_kernel<3072, 3>) and slice_finish_kernel; part = GN_PART_SLICES x npos
// x 16 int32 fc_0 partial sums, pinfo = npos (PSQT value, bucket) pairs (written by the plan),
// npos = n + the children;
// otherwise one launch over whole rows.  fin (optional): recorded after the stream launches
// (before the finish).  finish false (sliced stream): no slice_finish_kernel, out_parent /
// out_child stay unwritten: the caller's launch_finalize takes the big net's outputs from part
// and pinfo itself.
// phases: PLAN_PHASE (the pinfo reset and plan_kernel) and / or STREAM_PHASE (the stream launches
// and the finish), so that an expansion's plan can run on another stream than its row stream (the
// expansion pipeline, gpu_nnue.hip): the two calls take the same arguments.
constexpr int PLAN_PHASE = 1, STREAM_PHASE = 2;
hipError_t launch_plan_stream(const NetDevice &net, const gn_board *parents, size_t n, const uint64_t *offsets,
                              const ChildDelta *deltas, const uint8_t *need_parent, const uint8_t *need_child,
                              int2 *out_parent, int2 *out_child, int swz, const uint8_t *next_slot, int chain_k,
                              int kc, const uint64_t *eoff, uint64_t *ent, TileDesc *tiles, uint32_t *btiles,
                              uint32_t *pool, uint32_t *err, unsigned long long *rows_out,
                              unsigned long long *pads_out, size_t b0, size_t b1, const uint32_t *order,
                              hipEvent_t mid, hipStream_t s, int slices = 1, int32_t *part = nullptr,
                              size_t npos = 0, int2 *pinfo = nullptr, hipEvent_t fin = nullptr, bool finish = true,
                              int phases = PLAN_PHASE | STREAM_PHASE);
// GN_MODE_FULL preparation: need_small = valid && |simple_eval| > threshold,
// need_big = valid && !need_small.
hipError_t launch_classify(const gn_board *boards, size_t n, const gn_eval_params &P, uint8_t *need_small,
                           uint8_t *need_big, hipStream_t s);
// GN_MODE_FULL: marks need_big where the small net's |nnue| < reeval_threshold.
hipError_t launch_reeval(const int2 *out_small, const uint8_t *need_small, size_t n, const gn_eval_params &P,
                         uint8_t *need_big, hipStream_t s);
// Eval::evaluate epilogue -> gn_eval (flags incl. IN_CHECK / BAD_FEN).
// score: 0 child records (GN_FLAG_NO_SCORE); 1 positions: the score rule's static part
// (mate 0 / cp 0 without a legal move, from counts[i] when given, else found here; final_cp
// otherwise, which resolve_scores replaces for the in-check ones).
// owner / moves / unpacked (optional, children only): board i is unpacked[owner[i]] after
// moves[i] (the parents write_children unpacked), instead of unpacking boards[i].
// sliced (optional): the column-sliced stream's partial sums of the big net; position i's big-net
// output is then slice_finish_one of pinfo[qoff + i] (out_big[i] where pinfo.y < 0)
struct SlicedOut {
  const NetDevice *net;
  const int32_t *part;
  const int2 *pinfo;
  uint64_t npos, qoff;
};
hipError_t launch_finalize(const gn_board *boards, size_t n, int mode, const int2 *out_small,
                           const int2 *out_big, const uint8_t *need_small, const uint8_t *need_big,
                           const gn_eval_params &P, const Tables *tables, gn_eval *out, hipStream_t s,
                           int score, const uint64_t *counts = nullptr, const uint32_t *owner = nullptr,
                           const uint16_t *moves = nullptr, const Board *unpacked = nullptr,
                           const SlicedOut *sliced = nullptr);
// The score rule's in-check positions (include/gpu_nnue.h gn_eval.score): select (sel[n + 1],
// 1 for a scored position in check with a legal move), gather (idx / boards of the selected,
// pos = exclusive scan of sel), reduce (max over each selected position's replies
// [off[j], off[j + 1]) of moves / records ce, csv = the replies' own rule values where
// GN_FLAG_SEARCHED; writes score / flags / best_move of out[idx[j]] and sv[idx[j]] if sv).
hipError_t launch_score_select(const gn_eval *out, size_t n, uint64_t *sel, hipStream_t s);
hipError_t launch_score_gather(const gn_board *boards, const uint64_t *sel, const uint64_t *pos, size_t n,
                               uint32_t *idx, gn_board *sb, hipStream_t s);
// Replies already evaluated by an expansion (records rec / moves at [off[i], off[i + 1]) of
// parent i, the parents unpacked by write_children): compact offsets coff (m + 1, scan of
// counts; *total_host = coff[m], synchronous), then (_fill) ce / cb / cm = the selected
// parents' replies as positions of the rule (records with their static score part, boards,
// moves).
hipError_t launch_score_replies(const uint32_t *idx, size_t m, const uint64_t *off, uint64_t *counts,
                                uint64_t *coff, void *&temp, size_t &temp_bytes, uint64_t *total_host, hipStream_t s);
hipError_t launch_score_replies_fill(const uint32_t *idx, size_t m, const uint64_t *off, const uint64_t *coff,
                                     const gn_eval *rec, const uint16_t *moves, const Board *unpacked,
                                     const Tables *tables, gn_eval *ce, gn_board *cb, uint16_t *cm, hipStream_t s);
// (idx NULL: position j is sb[j] / out[j], and positions without replies are skipped)
hipError_t launch_score_reduce(const gn_board *sb, size_t m, const uint32_t *idx, const uint64_t *off,
                               const uint16_t *moves, const gn_eval *ce, const int32_t *csv, const gn_eval_params &P,
                               gn_eval *out, int32_t *sv, hipStream_t s);
// The small-batch graph's two reductions in one workgroup (idx NULL for both): level 1's positions
// sb1 [0, m1) from their replies (moves2 / ce2 / csv2 at off1) into out1 / sv1, then level 0's sb0
// [0, m0) from level 1's records and values (moves1 at off0) into out0.
hipError_t launch_score_reduce2(const gn_board *sb1, size_t m1, const uint64_t *off1, const uint16_t *moves2,
                                const gn_eval *ce2, const int32_t *csv2, gn_eval *out1, int32_t *sv1,
                                const gn_board *sb0, size_t m0, const uint64_t *off0, const uint16_t *moves1,
                                const gn_eval_params &P, gn_eval *out0, hipStream_t s);
// One level of the score rule's replies for a small batch in one launch (reply_level_kernel,
// kernels.hip): n <= 16,384 positions, selected from their boards (valid, in check, a legal move);
// replies into rb / rm [0, cap) (empty boards after the last), off = n + 1 offsets; *flag set
// (first) / or'd when the replies exceed cap.
hipError_t launch_reply_level(const gn_board *boards, size_t n, const Tables *tables, uint64_t *off, size_t cap,
                              gn_board *rb, uint16_t *rm, uint32_t *flag, int first, hipStream_t s);
// legal-move counts per board (invalid boards: 0); ebound (optional): per parent an
// upper bound of the planned expansion's list entries (stream.hip)
hipError_t launch_count_children(const gn_board *boards, size_t n, const Tables *tables, uint64_t *counts,
                                 hipStream_t s, uint64_t *ebound = nullptr);
// children of every board at offsets[i] (exclusive prefix sums of counts): their moves,
// owning board (owner, scratch) and, for children [c0, c0 + nc) (all children of these
// boards), the child boards, deltas and chained-walk links.  moves / owner: required.
// unpacked (optional, n entries): the boards unpacked once by the per-board pass, so that the
// per-child pass reads its parent instead of unpacking it again.
hipError_t launch_write_children(const gn_board *boards, size_t n, const Tables *tables, const uint64_t *offsets,
                                 size_t c0, size_t nc, gn_board *children, uint16_t *moves, uint32_t *owner,
                                 ChildDelta *deltas, uint8_t *next_slot, int chain_k, unsigned long long *rows,
                                 hipStream_t s, Board *unpacked = nullptr);
// sum of legal-move counts over all boards into *total (added; caller zeroes)
hipError_t launch_count_sum(const gn_board *boards, size_t n, const Tables *tables,
                            unsigned long long *total, hipStream_t s);
// random playouts (chess.h random_playout), one thread per position
hipError_t launch_random_positions(uint64_t seed, size_t first, size_t n, int max_plies, const Tables *tables,
                                   gn_board *out, hipStream_t s);
// random games: out[g * (plies + 1) + k] = position after k plies of game g
hipError_t launch_random_games(uint64_t seed, size_t first_game, size_t n_games, int plies, const Tables *tables,
                               gn_board *out, hipStream_t s);
// lichess batches replayed on the GPU: game g's move codes codes[moff[g], moff[g + 1]) from
// roots[g]; positions at boards[moff[g] + g + k], resolved moves at smoves[moff[g] + k - 1],
// status[g] = 0 or the 1-based index of the first illegal move (replay_games_kernel)
hipError_t launch_replay_games(const gn_board *roots, size_t ng, const uint64_t *moff, const uint16_t *codes,
                               const Tables *tables, gn_board *boards, uint16_t *smoves, int32_t *status, hipStream_t s);
// dst[i] = src[idx[i]]
hipError_t launch_gather_boards(const gn_board *src, const uint32_t *idx, size_t n, gn_board *dst, hipStream_t s);
// gn_eval -> gn_child (ABI v4 child records for the host-buffer calls)
hipError_t launch_pack_children(const gn_eval *in, size_t n, gn_child *out, hipStream_t s);
// narrowing copy of offsets for the C-ABI
hipError_t launch_offsets_u32(const uint64_t *in, size_t n, uint32_t *out, hipStream_t s);
// exclusive scan of n + 1 counts (counts[n] must be 0); temp grows on demand
hipError_t exclusive_scan_u64(const uint64_t *counts, uint64_t *offsets, size_t n1, void *&temp,
                              size_t &temp_bytes, hipStream_t s);

} // namespace gn
