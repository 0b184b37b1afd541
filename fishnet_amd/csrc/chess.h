// chess.h — bitboard chess core shared by host and device code of libgpu_nnue.
//
// Replaces, for the GPU path, what fishnet relies on the Stockfish process and
// shakmaty for:
//   - Position::set / FEN parsing with Chess960 castling (fishnet runs the
//     engine with UCI_Chess960 = true, /root/reference/src/stockfish.rs:200),
//   - legal move generation + do_move (children, perft),
//   - the packed 32-byte board that is the device input format (gn_board).
//
// Sliding attacks: hyperbola quintessence on full 64-bit bit reversal
// (v_bfrev_b32 on gfx950), one subtraction per line, no magics and no PEXT.
// The line / leaper masks (4 KiB, struct Tables) live in LDS inside kernels
// and in a static host copy for host callers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/gpu_nnue.h"

#define GN_HD __host__ __device__ __forceinline__

namespace gn {

typedef uint64_t Bitboard;
enum { WHITE = 0, BLACK = 1 };
enum { NO_PT = 0, PAWN = 1, KNIGHT = 2, BISHOP = 3, ROOK = 4, QUEEN = 5, KING = 6 };
enum { MT_NORMAL = 0, MT_PROMOTION = 1, MT_EN_PASSANT = 2, MT_CASTLING = 3 };
constexpr int SQ_NONE = 64;

GN_HD Bitboard sqbb(int s) { return 1ull << s; }
GN_HD int lsb(Bitboard b) { return __builtin_ctzll(b); }
GN_HD int popcnt(Bitboard b) { return __builtin_popcountll(b); }
GN_HD int pop_lsb(Bitboard &b) {
  int s = lsb(b);
  b &= b - 1;
  return s;
}
GN_HD Bitboard rbit(Bitboard b) { return __builtin_bitreverse64(b); }
GN_HD int make_piece(int c, int pt) { return (c << 3) | pt; }
GN_HD int rel_sq(int c, int s) { return c == WHITE ? s : s ^ 56; }

// line masks exclude the square itself: [0] file, [1] rank, [2] a1-h8 diagonal, [3] h1-a8 diagonal
struct Tables {
  Bitboard line[4][64];
  Bitboard knight[64];
  Bitboard king[64];
  Bitboard pawn[2][64]; // squares attacked by a pawn of colour c standing on s
};
static_assert(sizeof(Tables) == 4096, "tables are 4 KiB");

inline void init_tables(Tables &T) {
  for (int s = 0; s < 64; ++s) {
    int f = s & 7, r = s >> 3;
    Bitboard file = 0x0101010101010101ull << f, rank = 0xFFull << (8 * r), d = 0, a = 0;
    for (int k = -7; k <= 7; ++k) {
      if (f + k >= 0 && f + k < 8 && r + k >= 0 && r + k < 8) d |= sqbb((r + k) * 8 + f + k);
      if (f + k >= 0 && f + k < 8 && r - k >= 0 && r - k < 8) a |= sqbb((r - k) * 8 + f + k);
    }
    T.line[0][s] = file & ~sqbb(s);
    T.line[1][s] = rank & ~sqbb(s);
    T.line[2][s] = d & ~sqbb(s);
    T.line[3][s] = a & ~sqbb(s);
    static const int kn[8][2] = {{1, 2}, {2, 1}, {2, -1}, {1, -2}, {-1, -2}, {-2, -1}, {-2, 1}, {-1, 2}};
    Bitboard n = 0, k = 0;
    for (int i = 0; i < 8; ++i) {
      int nf = f + kn[i][0], nr = r + kn[i][1];
      if (nf >= 0 && nf < 8 && nr >= 0 && nr < 8) n |= sqbb(nr * 8 + nf);
    }
    for (int df = -1; df <= 1; ++df)
      for (int dr = -1; dr <= 1; ++dr) {
        int nf = f + df, nr = r + dr;
        if ((df || dr) && nf >= 0 && nf < 8 && nr >= 0 && nr < 8) k |= sqbb(nr * 8 + nf);
      }
    T.knight[s] = n;
    T.king[s] = k;
    Bitboard pw = 0, pb = 0;
    if (r < 7) {
      if (f > 0) pw |= sqbb(s + 7);
      if (f < 7) pw |= sqbb(s + 9);
    }
    if (r > 0) {
      if (f > 0) pb |= sqbb(s - 9);
      if (f < 7) pb |= sqbb(s - 7);
    }
    T.pawn[WHITE][s] = pw;
    T.pawn[BLACK][s] = pb;
  }
}

// hyperbola quintessence: attacks along one line with occupancy occ
GN_HD Bitboard line_attacks(Bitboard occ, int s, Bitboard mask) {
  Bitboard o = occ & mask;
  Bitboard f = o - sqbb(s);
  Bitboard r = rbit(rbit(o) - rbit(sqbb(s)));
  return (f ^ r) & mask;
}
GN_HD Bitboard rook_attacks(const Tables &T, int s, Bitboard occ) {
  return line_attacks(occ, s, T.line[0][s]) | line_attacks(occ, s, T.line[1][s]);
}
GN_HD Bitboard bishop_attacks(const Tables &T, int s, Bitboard occ) {
  return line_attacks(occ, s, T.line[2][s]) | line_attacks(occ, s, T.line[3][s]);
}
// squares strictly between a and b when aligned, else 0
GN_HD Bitboard between(const Tables &T, int a, int b) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (T.line[k][a] & sqbb(b)) return line_attacks(sqbb(b), a, T.line[k][a]) & line_attacks(sqbb(a), b, T.line[k][b]);
  return 0;
}
// full line through a and b (both included) when aligned, else 0
GN_HD Bitboard line_through(const Tables &T, int a, int b) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (T.line[k][a] & sqbb(b)) return T.line[k][a] | sqbb(a);
  return 0;
}

// Bitboard position.  byType[0] = all occupied squares.
struct Board {
  Bitboard byType[7];
  Bitboard byColor[2];
  uint8_t stm;
  uint8_t ep;             // SQ_NONE when none
  uint8_t castle_rook[4]; // [2c + 0] O-O rook square, [2c + 1] O-O-O rook square, SQ_NONE
  uint16_t rule50;
  uint16_t fullmove;
};

// Runtime-selected bitboards through unrolled constant indices only: keeps a
// Board in VGPRs on the device (no scratch) and can never index out of range.
// Each select mask is opaque to the optimiser, which would otherwise fold the
// constant-index updates back into one update at a runtime index and so move the
// whole Board to scratch memory (measured: 96 B/lane in the child kernel).
GN_HD Bitboard sel_mask(int t, int sel, Bitboard b) {
  Bitboard m = (t == sel) ? b : 0;
#ifdef __HIP_DEVICE_COMPILE__
  asm("" : "+v"(m));
#endif
  return m;
}
GN_HD Bitboard color_bb(const Board &B, int c) { return c ? B.byColor[1] : B.byColor[0]; }
GN_HD void xor_color(Board &B, int c, Bitboard b) {
  B.byColor[0] ^= sel_mask(0, c, b);
  B.byColor[1] ^= sel_mask(1, c, b);
}
GN_HD void or_color(Board &B, int c, Bitboard b) {
  B.byColor[0] |= sel_mask(0, c, b);
  B.byColor[1] |= sel_mask(1, c, b);
}
GN_HD void xor_type(Board &B, int pt, Bitboard b) {
#pragma unroll
  for (int t = PAWN; t <= KING; ++t) B.byType[t] ^= sel_mask(t, pt, b);
}
GN_HD void or_type(Board &B, int pt, Bitboard b) {
#pragma unroll
  for (int t = PAWN; t <= KING; ++t) B.byType[t] |= sel_mask(t, pt, b);
}

GN_HD int piece_on(const Board &B, int s) {
  Bitboard b = sqbb(s);
  if (!(B.byType[0] & b)) return 0;
  int c = (B.byColor[BLACK] & b) ? BLACK : WHITE;
  int pt = PAWN;
#pragma unroll
  for (int t = PAWN; t <= KING; ++t)
    if (B.byType[t] & b) pt = t;
  return make_piece(c, pt);
}

GN_HD Bitboard attackers_to(const Board &B, const Tables &T, int s, Bitboard occ) {
  return (T.pawn[BLACK][s] & B.byColor[WHITE] & B.byType[PAWN]) |
         (T.pawn[WHITE][s] & B.byColor[BLACK] & B.byType[PAWN]) | (T.knight[s] & B.byType[KNIGHT]) |
         (T.king[s] & B.byType[KING]) | (rook_attacks(T, s, occ) & (B.byType[ROOK] | B.byType[QUEEN])) |
         (bishop_attacks(T, s, occ) & (B.byType[BISHOP] | B.byType[QUEEN]));
}

GN_HD int king_square(const Board &B, int c) { return lsb(B.byType[KING] & color_bb(B, c)); }

GN_HD bool in_check(const Board &B, const Tables &T) {
  int us = B.stm;
  return (attackers_to(B, T, king_square(B, us), B.byType[0]) & color_bb(B, us ^ 1)) != 0;
}

// ------------------------------------------------------------- packing ----
// piece nibbles of a gn_board as two 64-bit words (nibble k of lo | hi << 64);
// avoids dynamic indexing into a register-resident byte array on the device
GN_HD void piece_words(const gn_board &p, uint64_t &lo, uint64_t &hi) {
  __builtin_memcpy(&lo, p.pc, 8);
  __builtin_memcpy(&hi, p.pc + 8, 8);
}
GN_HD int piece_nibble(uint64_t lo, uint64_t hi, int k) {
  return (int)(((k < 16 ? lo : hi) >> (4 * (k & 15))) & 15);
}

// Unpacks and validates a gn_board.  Returns false for anything the device
// must not touch (bad piece nibble, not exactly one king per side, > 32 pieces,
// pawns on a back rank, bad en-passant square).  Whether the side not to move
// is in check is NOT checked here.
GN_HD bool unpack(const gn_board &p, Board &B) {
  for (int i = 0; i < 7; ++i) B.byType[i] = 0;
  B.byColor[0] = B.byColor[1] = 0;
  Bitboard occ = p.occ;
  int n = popcnt(occ);
  if (n < 2 || n > 32) return false;
  bool ok = true;
  uint64_t wlo, whi;
  piece_words(p, wlo, whi);
  for (int k = 0; occ; ++k) {
    int s = pop_lsb(occ);
    int pc = piece_nibble(wlo, whi, k);
    int pt = pc & 7;
    ok &= pt >= PAWN && pt <= KING;
    or_type(B, pt, sqbb(s));
    or_color(B, pc >> 3, sqbb(s));
  }
  B.byType[0] = p.occ;
  ok &= popcnt(B.byType[KING] & B.byColor[WHITE]) == 1 && popcnt(B.byType[KING] & B.byColor[BLACK]) == 1;
  ok &= (B.byType[PAWN] & 0xFF000000000000FFull) == 0;
  B.stm = p.stm_ep >> 7;
  B.ep = p.stm_ep & 0x7F;
  if (B.ep > SQ_NONE) ok = false;
  for (int i = 0; i < 4; ++i) {
    int nib = (p.castle >> (4 * i)) & 15;
    B.castle_rook[i] = (nib & 8) ? (uint8_t)(((i >> 1) ? 56 : 0) + (nib & 7)) : (uint8_t)SQ_NONE;
  }
  B.rule50 = p.rule50;
  B.fullmove = p.fullmove;
  return ok;
}

GN_HD void pack(const Board &B, gn_board &p) {
  p.occ = B.byType[0];
  uint64_t lo = 0, hi = 0;
  Bitboard occ = B.byType[0];
  for (int k = 0; occ; ++k) {
    int s = pop_lsb(occ);
    uint64_t v = (uint64_t)piece_on(B, s) << (4 * (k & 15));
    if (k < 16) lo |= v;
    else hi |= v;
  }
  __builtin_memcpy(p.pc, &lo, 8);
  __builtin_memcpy(p.pc + 8, &hi, 8);
  p.stm_ep = (uint8_t)((B.stm << 7) | B.ep);
  p.reserved = 0;
  uint16_t c = 0;
  for (int i = 0; i < 4; ++i)
    if (B.castle_rook[i] != SQ_NONE) c |= (uint16_t)((8 | (B.castle_rook[i] & 7)) << (4 * i));
  p.castle = c;
  p.rule50 = B.rule50;
  p.fullmove = B.fullmove;
}

// --------------------------------------------------------------- moves ----
GN_HD uint16_t make_move(int from, int to, int type = MT_NORMAL, int promo = KNIGHT) {
  return (uint16_t)(to | (from << 6) | ((promo - KNIGHT) << 12) | (type << 14));
}
GN_HD int move_from(uint16_t m) { return (m >> 6) & 63; }
GN_HD int move_to(uint16_t m) { return m & 63; }
GN_HD int move_type(uint16_t m) { return m >> 14; }
GN_HD int move_promo(uint16_t m) { return ((m >> 12) & 3) + KNIGHT; }

// emit(m) of gen_legal returns void, or bool: true stops the generation (any_legal)
template <class F>
GN_HD bool emit_stop(F &emit, uint16_t m) {
  if constexpr (std::is_void<decltype(emit(m))>::value) {
    emit(m);
    return false;
  } else {
    return emit(m);
  }
}
#define GN_EMIT(m)                                                                                  \
  do {                                                                                              \
    if (emit_stop(emit, (m))) return;                                                               \
  } while (0)

// Legal move generator.  emit(uint16_t move) is called once per legal move,
// in a fixed order (king, knights, sliders, pawns, castling).
template <class F>
GN_HD void gen_legal(const Board &B, const Tables &T, F &&emit) {
  const int us = B.stm, them = us ^ 1;
  const Bitboard occ = B.byType[0], ours = color_bb(B, us), theirs = color_bb(B, them);
  const int ksq = king_square(B, us);
  const Bitboard checkers = attackers_to(B, T, ksq, occ) & theirs;
  // king
  {
    Bitboard tg = T.king[ksq] & ~ours, occ_nok = occ ^ sqbb(ksq);
    while (tg) {
      int to = pop_lsb(tg);
      if (!(attackers_to(B, T, to, occ_nok) & theirs)) GN_EMIT(make_move(ksq, to));
    }
  }
  if (checkers & (checkers - 1)) return; // double check: king moves only
  // pinned pieces
  Bitboard pinned = 0;
  {
    Bitboard rq = (B.byType[ROOK] | B.byType[QUEEN]) & theirs, bq = (B.byType[BISHOP] | B.byType[QUEEN]) & theirs;
    Bitboard snipers = ((T.line[0][ksq] | T.line[1][ksq]) & rq) | ((T.line[2][ksq] | T.line[3][ksq]) & bq);
    while (snipers) {
      int s = pop_lsb(snipers);
      Bitboard b = between(T, ksq, s) & occ;
      if (b && !(b & (b - 1)) && (b & ours)) pinned |= b;
    }
  }
  const Bitboard target = checkers ? (between(T, ksq, lsb(checkers)) | checkers) : ~ours;
  // knights (a pinned knight never moves)
  {
    Bitboard pcs = B.byType[KNIGHT] & ours & ~pinned;
    while (pcs) {
      int from = pop_lsb(pcs);
      Bitboard tg = T.knight[from] & target;
      while (tg) GN_EMIT(make_move(from, pop_lsb(tg)));
    }
  }
  // sliders
  {
    Bitboard pcs = (B.byType[BISHOP] | B.byType[ROOK] | B.byType[QUEEN]) & ours;
    while (pcs) {
      int from = pop_lsb(pcs);
      Bitboard f = sqbb(from), att = 0;
      if (f & (B.byType[ROOK] | B.byType[QUEEN])) att |= rook_attacks(T, from, occ);
      if (f & (B.byType[BISHOP] | B.byType[QUEEN])) att |= bishop_attacks(T, from, occ);
      att &= target;
      if (pinned & f) att &= line_through(T, ksq, from);
      while (att) GN_EMIT(make_move(from, pop_lsb(att)));
    }
  }
  // pawns
  {
    const int up = us == WHITE ? 8 : -8;
    const Bitboard last = us == WHITE ? 0xFF00000000000000ull : 0xFFull;
    const Bitboard start = us == WHITE ? 0xFF00ull : 0xFF000000000000ull;
    Bitboard pcs = B.byType[PAWN] & ours;
    while (pcs) {
      int from = pop_lsb(pcs);
      Bitboard f = sqbb(from), allowed = (pinned & f) ? line_through(T, ksq, from) : ~0ull;
      Bitboard tg = 0;
      int one = from + up;
      if (!(occ & sqbb(one))) {
        tg |= sqbb(one);
        if ((f & start) && !(occ & sqbb(one + up))) tg |= sqbb(one + up);
      }
      tg |= T.pawn[us][from] & theirs;
      tg &= target & allowed;
      while (tg) {
        int to = pop_lsb(tg);
        if (sqbb(to) & last) {
          GN_EMIT(make_move(from, to, MT_PROMOTION, QUEEN));
          GN_EMIT(make_move(from, to, MT_PROMOTION, ROOK));
          GN_EMIT(make_move(from, to, MT_PROMOTION, BISHOP));
          GN_EMIT(make_move(from, to, MT_PROMOTION, KNIGHT));
        } else
          GN_EMIT(make_move(from, to));
      }
      if (B.ep != SQ_NONE && (T.pawn[us][from] & sqbb(B.ep))) {
        // full simulation: removes both pawns, adds ours on ep, recomputes attackers
        int cap = B.ep - up;
        Bitboard occ2 = (occ ^ f ^ sqbb(cap)) | sqbb(B.ep);
        Bitboard th2 = theirs ^ sqbb(cap);
        Bitboard att = ((rook_attacks(T, ksq, occ2) & (B.byType[ROOK] | B.byType[QUEEN])) |
                        (bishop_attacks(T, ksq, occ2) & (B.byType[BISHOP] | B.byType[QUEEN])) |
                        (T.knight[ksq] & B.byType[KNIGHT]) | (T.pawn[us][ksq] & B.byType[PAWN])) &
                       th2;
        if (!att) GN_EMIT(make_move(from, B.ep, MT_EN_PASSANT));
      }
    }
  }
  // castling (Chess960 rules; generated only when not in check)
  if (!checkers) {
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      int rsq = us ? B.castle_rook[2 + side] : B.castle_rook[side];
      if (rsq == SQ_NONE) continue;
      if (!(B.byType[ROOK] & ours & sqbb(rsq))) continue;
      int kto = rel_sq(us, side == 0 ? 6 : 2), rto = rel_sq(us, side == 0 ? 5 : 3);
      Bitboard kpath = between(T, ksq, kto) | sqbb(kto), rpath = between(T, rsq, rto) | sqbb(rto);
      if ((kpath | rpath) & occ & ~sqbb(ksq) & ~sqbb(rsq)) continue;
      Bitboard walk = kto == ksq ? 0 : kpath;
      bool ok = true;
      while (walk && ok) ok = !(attackers_to(B, T, pop_lsb(walk), occ) & theirs);
      if (!ok) continue;
      Bitboard occ2 = (occ ^ sqbb(ksq) ^ sqbb(rsq)) | sqbb(kto) | sqbb(rto);
      Bitboard sl = ((rook_attacks(T, kto, occ2) & (B.byType[ROOK] | B.byType[QUEEN])) |
                     (bishop_attacks(T, kto, occ2) & (B.byType[BISHOP] | B.byType[QUEEN]))) &
                    theirs;
      if (sl) continue;
      GN_EMIT(make_move(ksq, rsq, MT_CASTLING));
    }
  }
}

// What a move changes, for incremental feature-transformer updates.
struct Dirty {
  int n_rem, n_add;
  int rem_sq[2], rem_pc[2]; // mover at from (or king at from for castling), captured piece
  int add_sq[2], add_pc[2]; // mover / promoted piece at to, rook at rto
  bool king_moved;          // mover's perspective needs a refresh
};

GN_HD Board do_move(const Board &B, uint16_t m, Dirty *d = nullptr) {
  Board C = B;
  const int us = B.stm, them = us ^ 1;
  const int from = move_from(m), to = move_to(m), type = move_type(m);
  const int pc = piece_on(B, from), pt = pc & 7;
  const int ksq = king_square(B, us);
  int captured = 0;
  if (d) d->n_rem = d->n_add = 0, d->king_moved = pt == KING;
  if (type == MT_CASTLING) {
    int kside = to > from;
    int kto = rel_sq(us, kside ? 6 : 2), rto = rel_sq(us, kside ? 5 : 3);
    C.byType[KING] ^= sqbb(from) ^ sqbb(kto); // no-op when the king stays (kto == from)
    C.byType[ROOK] ^= sqbb(to) ^ sqbb(rto);   // no-op when the rook stays (rto == to)
    xor_color(C, us, sqbb(from) | sqbb(to));
    or_color(C, us, sqbb(kto) | sqbb(rto));
    C.byType[0] = C.byColor[0] | C.byColor[1];
    if (d) {
      d->n_rem = 2, d->rem_sq[0] = from, d->rem_pc[0] = make_piece(us, KING), d->rem_sq[1] = to,
      d->rem_pc[1] = make_piece(us, ROOK);
      d->n_add = 2, d->add_sq[0] = kto, d->add_pc[0] = make_piece(us, KING), d->add_sq[1] = rto,
      d->add_pc[1] = make_piece(us, ROOK);
    }
  } else {
    int capsq = type == MT_EN_PASSANT ? to - (us == WHITE ? 8 : -8) : to;
    captured = piece_on(B, capsq);
    if (captured) {
      xor_type(C, captured & 7, sqbb(capsq));
      xor_color(C, them, sqbb(capsq));
    }
    int newpt = type == MT_PROMOTION ? move_promo(m) : pt;
    xor_type(C, pt, sqbb(from));
    or_type(C, newpt, sqbb(to));
    xor_color(C, us, sqbb(from) | sqbb(to));
    C.byType[0] = C.byColor[0] | C.byColor[1];
    if (d) {
      d->rem_sq[0] = from, d->rem_pc[0] = pc, d->n_rem = 1;
      if (captured) d->rem_sq[1] = capsq, d->rem_pc[1] = captured, d->n_rem = 2;
      d->add_sq[0] = to, d->add_pc[0] = make_piece(us, newpt), d->n_add = 1;
    }
  }
  C.rule50 = (type != MT_CASTLING && (pt == PAWN || captured)) ? 0 : (B.rule50 < 65535 ? B.rule50 + 1 : 65535);
  C.ep = SQ_NONE;
  if (pt == PAWN && (to ^ from) == 16) {
    // ep square only when an enemy pawn stands beside the pushed pawn (it can capture)
    Bitboard adj = ((sqbb(to) << 1) & ~0x0101010101010101ull) | ((sqbb(to) >> 1) & ~0x8080808080808080ull);
    if (adj & B.byType[PAWN] & color_bb(B, them)) C.ep = (uint8_t)((from + to) / 2);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r = C.castle_rook[i];
    if (r == SQ_NONE) continue;
    if (r == from || r == to || ((i >> 1) == us && from == ksq)) C.castle_rook[i] = SQ_NONE;
  }
  if (us == BLACK && C.fullmove < 65535) C.fullmove++;
  C.stm = (uint8_t)them;
  return C;
}

// ------------------------------------------------------------- UCI moves ----
// A lichess move token (AcquireResponseBody.moves, /root/reference/src/api.rs:306-321) as a
// 16-bit code: from | to << 6 | promo << 12 (promo 0 none, 1..4 = n b r q); UCI_BAD for a
// token that is not from-square + to-square (+ promotion letter).
constexpr uint16_t UCI_BAD = 0xFFFF;
GN_HD uint16_t uci_code(const char *u, int len) {
  if (len != 4 && len != 5) return UCI_BAD;
  if (u[0] < 'a' || u[0] > 'h' || u[1] < '1' || u[1] > '8' || u[2] < 'a' || u[2] > 'h' || u[3] < '1' || u[3] > '8')
    return UCI_BAD;
  int promo = 0;
  if (len == 5) {
    promo = u[4] == 'n' ? 1 : u[4] == 'b' ? 2 : u[4] == 'r' ? 3 : u[4] == 'q' ? 4 : -1;
    if (promo < 0) return UCI_BAD;
  }
  const int from = (u[1] - '1') * 8 + (u[0] - 'a'), to = (u[3] - '1') * 8 + (u[2] - 'a');
  return (uint16_t)(from | to << 6 | promo << 12);
}

// shakmaty 0.27.3 UciMove::to_move (the reference's move resolution, queue.rs:576), standard
// chess: the king moving onto a square of the castling rights is castling with that rook
// (Chess960 notation, king takes rook); the king moving from e1/e8 to the c/g file of its
// back rank is castling with the a/h rook (standard notation); otherwise the move from
// `from` to `to` (en passant included) with the promotion piece; the candidate must be
// legal.  Host (gn_replay_game) and device (the GPU replay of gn_evaluate_games) run this.
GN_HD bool resolve_uci(const Board &B, const Tables &T, uint16_t code, uint16_t &out) {
  if (code == UCI_BAD) return false;
  const int from = code & 63, to = (code >> 6) & 63, pr = code >> 12;
  const int promo = pr ? KNIGHT + pr - 1 : 0;
  const int pc = piece_on(B, from);
  if (!pc || (promo && (pc & 7) != PAWN)) return false;
  const int us = B.stm;
  int rook = -1;
  if ((pc & 7) == KING) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (B.castle_rook[i] == to) rook = to;
    if (rook < 0 && from == (us ? 60 : 4) && (to >> 3) == (us ? 7 : 0) && ((to & 7) == 2 || (to & 7) == 6))
      rook = (to & 56) | ((to & 7) == 2 ? 0 : 7);
  }
  bool found = false;
  gen_legal(B, T, [&](uint16_t m) {
    if (move_from(m) != from) return false;
    const int t = move_type(m);
    if (rook >= 0) {
      if (t == MT_CASTLING && move_to(m) == rook) found = true, out = m;
      return found;
    }
    if (t == MT_CASTLING || move_to(m) != to) return false;
    if (t == MT_PROMOTION ? move_promo(m) != promo : promo != 0) return false;
    found = true, out = m;
    return true;
  });
  return found;
}

// ------------------------------------------------------ random playouts ----
// xoshiro256** (Blackman & Vigna), seeded through splitmix64
struct Xoshiro {
  uint64_t s0, s1, s2, s3;
  GN_HD explicit Xoshiro(uint64_t seed) {
    s0 = mix(seed += 0x9E3779B97F4A7C15ull);
    s1 = mix(seed += 0x9E3779B97F4A7C15ull);
    s2 = mix(seed += 0x9E3779B97F4A7C15ull);
    s3 = mix(seed += 0x9E3779B97F4A7C15ull);
  }
  GN_HD static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  GN_HD static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  GN_HD uint64_t next() {
    uint64_t r = rotl(s1 * 5, 7) * 9, t = s1 << 17;
    s2 ^= s0, s3 ^= s1, s1 ^= s2, s0 ^= s3, s2 ^= t, s3 = rotl(s3, 45);
    return r;
  }
  GN_HD uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * n >> 32); }
};

GN_HD Board start_position() {
  Board B;
  B.byType[PAWN] = 0x00FF00000000FF00ull;
  B.byType[KNIGHT] = 0x4200000000000042ull;
  B.byType[BISHOP] = 0x2400000000000024ull;
  B.byType[ROOK] = 0x8100000000000081ull;
  B.byType[QUEEN] = 0x0800000000000008ull;
  B.byType[KING] = 0x1000000000000010ull;
  B.byColor[WHITE] = 0xFFFFull;
  B.byColor[BLACK] = 0xFFFF000000000000ull;
  B.byType[0] = B.byColor[WHITE] | B.byColor[BLACK];
  B.stm = WHITE, B.ep = SQ_NONE;
  B.castle_rook[0] = 7, B.castle_rook[1] = 0, B.castle_rook[2] = 63, B.castle_rook[3] = 56;
  B.rule50 = 0, B.fullmove = 1;
  return B;
}

// any legal move (stalemate / checkmate detection): stops at the first one
GN_HD bool any_legal(const Board &B, const Tables &T) {
  bool any = false;
  gen_legal(B, T, [&](uint16_t) {
    any = true;
    return true;
  });
  return any;
}

GN_HD int count_legal(const Board &B, const Tables &T) {
  int n = 0;
  gen_legal(B, T, [&](uint16_t) { ++n; });
  return n;
}

GN_HD uint16_t nth_legal(const Board &B, const Tables &T, int r) {
  uint16_t pick = 0;
  int k = 0;
  gen_legal(B, T, [&](uint16_t m) {
    if (k++ == r) pick = m;
  });
  return pick;
}

// Random playout from the start position (SURVEY.md §8d workload): k ~
// U{0..max_plies} uniformly random legal plies, stopping at mate / stalemate /
// rule50 >= 100; a final position in check is played on (<= 8 plies) or the
// playout restarts (bounded: 64 attempts).  Host and device run this same code,
// so a seed gives the same position everywhere.
GN_HD Board random_playout(uint64_t seed, int max_plies, const Tables &T) {
  Xoshiro rng(seed);
  Board B = start_position();
  for (int attempt = 0; attempt < 64; ++attempt) {
    B = start_position();
    const int k = (int)rng.below((uint32_t)max_plies + 1);
    for (int ply = 0; ply < k; ++ply) {
      const int n = count_legal(B, T);
      if (!n || B.rule50 >= 100) break;
      B = do_move(B, nth_legal(B, T, (int)rng.below((uint32_t)n)));
    }
    for (int extra = 0; extra < 8 && in_check(B, T); ++extra) {
      const int n = count_legal(B, T);
      if (!n) break;
      B = do_move(B, nth_legal(B, T, (int)rng.below((uint32_t)n)));
    }
    if (!in_check(B, T)) break;
  }
  return B;
}

// A random game (the bench's lichess-shaped batches): `plies` uniformly random legal plies
// from the start position (xoshiro256**, seed); emit(k, B, move) for k = 0..plies with the
// position after k plies and the move that made it (0 for k = 0, and for the plies after the
// game ended: mate, stalemate or rule50 >= 100 repeat the final position).
template <class F>
GN_HD void random_game(uint64_t seed, int plies, const Tables &T, F &&emit) {
  Xoshiro rng(seed);
  Board B = start_position();
  emit(0, B, (uint16_t)0);
  for (int k = 1; k <= plies; ++k) {
    const int n = count_legal(B, T);
    uint16_t m = 0;
    if (n && B.rule50 < 100) {
      m = nth_legal(B, T, (int)rng.below((uint32_t)n));
      B = do_move(B, m);
    }
    emit(k, B, m);
  }
}

// UCI text of a move in Stockfish encoding as the lichess API sends it (standard chess:
// castling as the king's two-square move, e1g1; Chess960 positions: king takes rook);
// buf >= 6 bytes; returns the length.
GN_HD int move_uci(uint16_t m, char *buf) {
  int from = move_from(m), to = move_to(m);
  if (move_type(m) == MT_CASTLING && (from == 4 || from == 60) && ((to & 7) == 0 || (to & 7) == 7))
    to = (to & 56) | ((to & 7) == 0 ? 2 : 6);
  buf[0] = (char)('a' + (from & 7)), buf[1] = (char)('1' + (from >> 3));
  buf[2] = (char)('a' + (to & 7)), buf[3] = (char)('1' + (to >> 3));
  int n = 4;
  if (move_type(m) == MT_PROMOTION) buf[n++] = "nbrq"[move_promo(m) - KNIGHT];
  buf[n] = '\0';
  return n;
}

} // namespace gn
