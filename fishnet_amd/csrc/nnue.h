// nnue.h — Stockfish NNUE (HalfKAv2_hm, SF 17.1-era) as laid out in HBM by
// libgpu_nnue, shared between the host loader and the kernels.
//
// HBM layout of one network (all arrays 256-B aligned):
//   ft      [22528 + 1][RS] bytes, RS = 2*L1 + 32 rounded up to 128: one feature's
//           row is the L1 int16 feature-transformer weights (doubled at load, as
//           Stockfish scale_weights does) followed by its 8 int32 PSQT weights, so
//           one gathered feature = one contiguous row (6,272 B big / 384 B small;
//           the 128-B start keeps the L1 weights on 48 whole lines, not 49).
//           Row FT_BIAS_ROW (the extra last row) is the bias with zero PSQT, so
//           a refresh is "zero + bias row + feature rows" in one row stream.
//   bias    [L1] int16 (doubled)
//   w0      [8 buckets][16][L1] int8     b0 [8][16] int32    (fc_0)
//   w1      [8][32][32] int8             b1 [8][32] int32    (fc_1, cols 30,31 pad)
//   w2      [8][32] int8                 b2 [8] int32        (fc_2)
//   psqt    [8 buckets][22528 + 1] int32: the PSQT weights again, bucket-major (L2-sized)
//   w0f     [8][L1 / 64][64][16] int8: w0 again, one 1 KiB block per 64-wide k-step in the
//           operand order of v_mfma_i32_16x16x64_i8 (lane l: output l & 15, inputs 16 (l >> 4) ..)
#pragma once
#include <stdint.h>

#include "chess.h"

namespace gn {

constexpr int FT_INPUTS = 22528;
constexpr int FT_BIAS_ROW = FT_INPUTS; // see the layout above
constexpr int FT_ROWS = FT_INPUTS + 1;
// FT row stride in bytes: 2*L1 + 32 rounded up to GN_ROW_ALIGN (a 128-B multiple keeps a
// row's L1 weights on whole 128-B lines)
#ifndef GN_ROW_ALIGN
#define GN_ROW_ALIGN 128
#endif
constexpr uint32_t ft_row_stride(uint32_t l1) { return (2 * l1 + 32 + GN_ROW_ALIGN - 1) / GN_ROW_ALIGN * GN_ROW_ALIGN; }
// Big nets: CARRY_SLOTS x 132 scratch rows follow the FT rows in the same allocation
// (round 1's chained walk had 4 carry rows + 128 king-cache rows per slot; the planned
// expansion's scratch slots below use the same rows).  Row indices stay below 2^19 (the
// row field of a stream entry).
constexpr int CARRY_SLOTS = 2048;
constexpr int CARRY_ROW0 = FT_ROWS;
// Then the king cache: per slot, one accumulator row per (perspective, king square).
constexpr int KC_ROW0 = CARRY_ROW0 + 4 * CARRY_SLOTS;
static_assert(KC_ROW0 + 128 * CARRY_SLOTS <= (1 << 19), "carry and king-cache rows must fit the 19-bit row field");
// The planned expansion (stream.hip) gives each running workgroup a scratch slot of
// SCR_ROWS rows from a pool of POOL_PER_XCD slots per XCD: rows 2 + 64 h + ksq are the
// king-cache rows (perspective x king square); rows 0 and 1 are unused since its chained
// walk carries the next parent in registers.  The slots occupy the same rows behind the
// FT rows as the carry / king-cache rows above.
constexpr int SCR_ROWS = 130;
constexpr int POOL_PER_XCD = 256;
constexpr int SCR_SLOTS = 8 * POOL_PER_XCD;
static_assert(SCR_ROWS * SCR_SLOTS <= 132 * CARRY_SLOTS, "scratch slots fit the rows behind the FT rows");
// One row of zeros after all of those (never written): the row a store-only stream entry
// loads, so that its multiplier may carry the store's target row (stream.hip).
constexpr int ZERO_ROW = FT_ROWS + 132 * CARRY_SLOTS;
static_assert(ZERO_ROW < (1 << 19), "the zero row fits the 19-bit row field");
constexpr int PSQT_BUCKETS = 8;
constexpr int LAYER_STACKS = 8;
constexpr uint32_t NNUE_VERSION = 0x7AF32F20u;

struct NetDevice {
  int L1;
  uint32_t row_stride;
  int carry_slots; // CARRY_SLOTS when the carry rows exist (big nets), else 0
  int kc_slots;    // CARRY_SLOTS when the king-cache rows exist (big nets), else 0
  const uint8_t *ft;
  const int16_t *bias;
  const int8_t *w0;
  const int32_t *b0;
  const int8_t *w1;
  const int32_t *b1;
  const int8_t *w2;
  const int32_t *b2;
  const int32_t *psqt; // [PSQT_BUCKETS][FT_ROWS]: the rows' PSQT weights by bucket (a copy)
  const int8_t *w0f;   // [8][L1 / 64][64 lanes][16]: w0 in the int8 MFMA's operand order (a copy)
};

// HalfKAv2_hm feature index:
//   (sq ^ orient) + 64 * plane(piece, perspective) + 704 * king_bucket
// orient mirrors files when the perspective's king is on files a-d and flips
// ranks for black; king_bucket = 4 * (7 - relative rank) + min(file, 7 - file);
// planes: own P N B R Q = 0 2 4 6 8, their P N B R Q = 1 3 5 7 9, kings = 10.
GN_HD int feature_index(int persp, int sq, int pc, int ksq) {
  const int kf = ksq & 7;
  const int orient = (kf < 4 ? 7 : 0) ^ (persp ? 56 : 0);
  const int rel_rank = (ksq >> 3) ^ (persp ? 7 : 0);
  const int bucket = 4 * (7 - rel_rank) + (kf < 4 ? kf : 7 - kf);
  const int pt = pc & 7;
  const int plane = pt == KING ? 10 : 2 * (pt - 1) + ((pc >> 3) != persp);
  return (sq ^ orient) + 64 * plane + 704 * bucket;
}

// Feature-transformer delta of one child, written by the child generator
// (write_children) from Dirty and read by expand_eval: for each ABSOLUTE
// perspective either a refresh flag or up to 2 removed (idx[h][0..1]) and 2
// added (idx[h][2..3]) HalfKAv2_hm rows.
struct ChildDelta {
  uint16_t idx[2][4];
  uint32_t meta; // [1:0] nsub w, [3:2] nadd w, [5:4] nsub b, [7:6] nadd b, [8] refresh w, [9] refresh b,
                 // [10] stm, [13:11] bucket, [19:14] child piece count
  uint32_t pad;
};
static_assert(sizeof(ChildDelta) == 24, "ChildDelta is 24 bytes");

GN_HD ChildDelta make_child_delta(const Board &parent, const Board &child, const Dirty &d) {
  ChildDelta cd;
  uint32_t meta = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ksq = king_square(child, h);
    cd.idx[h][0] = cd.idx[h][1] = cd.idx[h][2] = cd.idx[h][3] = 0;
    if (d.king_moved && h == parent.stm) {
      // refresh of the mover's perspective: the squares that change instead of rows
      // (king from, king to, and for castling rook from, rook to; 64 = none), so the
      // evaluator derives the child's features from the parent board
      meta |= 1u << (8 + h);
      const bool castle = d.n_add == 2; // castling: king + rook moved
      cd.idx[h][0] = (uint16_t)d.rem_sq[0];
      cd.idx[h][1] = (uint16_t)d.add_sq[0];
      cd.idx[h][2] = (uint16_t)(castle ? d.rem_sq[1] : 64);
      cd.idx[h][3] = (uint16_t)(castle ? d.add_sq[1] : 64);
    } else {
      cd.idx[h][0] = (uint16_t)feature_index(h, d.rem_sq[0], d.rem_pc[0], ksq);
      if (d.n_rem > 1) cd.idx[h][1] = (uint16_t)feature_index(h, d.rem_sq[1], d.rem_pc[1], ksq);
      cd.idx[h][2] = (uint16_t)feature_index(h, d.add_sq[0], d.add_pc[0], ksq);
      if (d.n_add > 1) cd.idx[h][3] = (uint16_t)feature_index(h, d.add_sq[1], d.add_pc[1], ksq);
      meta |= (uint32_t)(d.n_rem | (d.n_add << 2)) << (4 * h);
    }
  }
  meta |= (uint32_t)child.stm << 10;
  meta |= (uint32_t)((popcnt(child.byType[0]) - 1) / 4) << 11;
  meta |= (uint32_t)popcnt(child.byType[0]) << 14;
  cd.meta = meta;
  cd.pad = 0;
  return cd;
}

// Feature rows of both absolute perspectives straight from a packed board
// (no Board needed).  Returns the piece count, or 0 for an invalid board
// (bad nibble, not one king per side): nothing is then written, so no row
// index can go out of range.
GN_HD int packed_features(const gn_board &p, uint16_t *rows_white, uint16_t *rows_black) {
  uint64_t wlo, whi;
  piece_words(p, wlo, whi);
  const int c = popcnt(p.occ);
  int wk = -1, bk = -1;
  bool ok = c >= 2 && c <= 32;
  uint64_t o = p.occ;
  for (int k = 0; ok && k < c; ++k) {
    const int s = pop_lsb(o), pc = piece_nibble(wlo, whi, k), pt = pc & 7;
    ok &= pt >= PAWN && pt <= KING;
    if (pc == make_piece(WHITE, KING)) ok &= wk < 0, wk = s;
    if (pc == make_piece(BLACK, KING)) ok &= bk < 0, bk = s;
  }
  if (!ok || wk < 0 || bk < 0) return 0;
  o = p.occ;
  for (int k = 0; k < c; ++k) {
    const int s = pop_lsb(o), pc = piece_nibble(wlo, whi, k);
    if (rows_white) rows_white[k] = (uint16_t)feature_index(WHITE, s, pc, wk);
    if (rows_black) rows_black[k] = (uint16_t)feature_index(BLACK, s, pc, bk);
  }
  return c;
}

// UCIEngine::to_cp (Stockfish 17-era uci.cpp, SURVEY.md §8a row a18, recalled):
// a = p_a(m) of the win-rate model, m = clamp(material, lo, hi) / anchor, and
// cp = round(100 * v / a).  Evaluated in double in Stockfish's operation order
// with contraction off (Stockfish's gcc -std=c++17 build does not fuse), rounded
// half away from zero as std::round; saturated to int32 (0 for a non-finite quotient).
GN_HD int wdl_material(const Board &B, const gn_eval_params &P) {
  int m = 0;
#pragma unroll
  for (int pt = PAWN; pt <= QUEEN; ++pt) m += P.wdl_piece_weight[pt - 1] * popcnt(B.byType[pt]);
  return m;
}
GN_HD int32_t wdl_to_cp(int32_t v, int material, const gn_eval_params &P) {
#pragma clang fp contract(off)
  const int lo = P.wdl_material_min, hi = P.wdl_material_max;
  const int mc = material < lo ? lo : material > hi ? hi : material;
  const double m = (double)mc / (double)P.wdl_material_anchor;
  const double a = ((P.wdl_a[0] * m + P.wdl_a[1]) * m + P.wdl_a[2]) * m + P.wdl_a[3];
  const double cp = round((double)(100 * (int64_t)v) / a);
  if (!(cp == cp)) return 0;
  return cp > 2147483647.0 ? 2147483647 : cp < -2147483647.0 ? -2147483647 : (int32_t)cp;
}

// ---- the score rule (gn_eval.score, include/gpu_nnue.h) --------------------------------
// Values in Stockfish's units: VALUE_MATE - ply for a mate ply plies away, static
// evaluations clamped below VALUE_MATE_IN_MAX_PLY (gn_eval_params.value_clamp).
constexpr int32_t VALUE_MATE = 32000, VALUE_MATE_IN_MAX_PLY = 32000 - 246;
// The value a record contributes to its parent's in-check rule (its side-to-move POV);
// `searched` is its own rule value when GN_FLAG_SEARCHED is set.
GN_HD int32_t rule_value(uint32_t flags, int32_t final_v, int32_t searched) {
  if (flags & GN_FLAG_NO_MOVES) return (flags & GN_FLAG_IN_CHECK) ? -VALUE_MATE : 0;
  return (flags & GN_FLAG_SEARCHED) ? searched : final_v;
}
// A reply's value seen from the position before it: negated, mates one ply further away.
GN_HD int32_t negate_ply(int32_t v) {
  v = -v;
  return v >= VALUE_MATE_IN_MAX_PLY ? v - 1 : v <= -VALUE_MATE_IN_MAX_PLY ? v + 1 : v;
}
// score / GN_FLAG_MATE of a rule value, as Stockfish's UCI `score` prints it
// (mate (ply + 1) / 2 when mating, -ply / 2 when mated; else cp by to_cp).
GN_HD int32_t rule_score(int32_t v, int material, const gn_eval_params &P, uint32_t &flags) {
  if (v >= VALUE_MATE_IN_MAX_PLY || v <= -VALUE_MATE_IN_MAX_PLY) {
    const int32_t ply = VALUE_MATE - (v > 0 ? v : -v);
    flags |= GN_FLAG_MATE;
    return v > 0 ? (ply + 1) / 2 : -ply / 2;
  }
  return wdl_to_cp(v, material, P);
}

// 32-bit hashes stored in .nnue files
inline uint32_t affine_hash(uint32_t prev, uint32_t outs) {
  uint32_t h = 0xCC03DAE4u + outs;
  h ^= prev >> 1;
  h ^= prev << 31;
  return h;
}
inline uint32_t ft_hash(int l1) { return 0x7f234cb8u ^ (uint32_t)(l1 * 2); }
inline uint32_t arch_hash(int l1) {
  uint32_t h = 0xEC42E90Du ^ (uint32_t)(l1 * 2);
  h = affine_hash(h, 16);
  h = 0x538D24C7u + h;
  h = affine_hash(h, 32);
  h = 0x538D24C7u + h;
  return affine_hash(h, 1);
}

} // namespace gn
