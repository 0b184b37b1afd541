// host_board.h — host-only board utilities of libgpu_nnue: FEN <-> Board,
// random-playout workload generator.
//
// FEN semantics mirror what the reference feeds Stockfish: shakmaty FENs
// (X-FEN castling, en passant only when legal — /root/reference/src/queue.rs:570)
// parsed with UCI_Chess960 = true (/root/reference/src/stockfish.rs:200), i.e.
// Stockfish's Position::set castling rules: K/Q pick the outermost rook on that
// side, A-H name the rook file (Shredder-FEN / X-FEN).
#pragma once
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "chess.h"

namespace gn {

const Tables &host_tables();

inline int piece_from_char(char c) {
  const char *w = "PNBRQK", *b = "pnbrqk";
  for (int i = 0; i < 6; ++i) {
    if (c == w[i]) return make_piece(WHITE, i + 1);
    if (c == b[i]) return make_piece(BLACK, i + 1);
  }
  return 0;
}

inline void put_piece(Board &B, int s, int pc) {
  or_type(B, pc & 7, sqbb(s));
  or_color(B, pc >> 3, sqbb(s));
  B.byType[0] |= sqbb(s);
}

// Returns true on success.  Rejects: malformed placement, not exactly one king
// per side, more than 32 pieces, pawns on the first/last rank, side not to move
// in check.  Missing trailing fields default to "w - - 0 1".
inline bool parse_fen(const char *fen, Board &B) {
  const Tables &T = host_tables();
  memset(&B, 0, sizeof(B));
  B.ep = SQ_NONE;
  for (int i = 0; i < 4; ++i) B.castle_rook[i] = SQ_NONE;
  B.fullmove = 1;
  if (!fen) return false;
  const char *s = fen;
  while (*s == ' ') ++s;
  int rank = 7, file = 0;
  while (*s && *s != ' ') {
    char c = *s++;
    if (c == '/') {
      if (file != 8 || rank == 0) return false;
      --rank, file = 0;
    } else if (c >= '1' && c <= '8') {
      file += c - '0';
      if (file > 8) return false;
    } else {
      int pc = piece_from_char(c);
      if (!pc || file > 7) return false;
      put_piece(B, rank * 8 + file++, pc);
    }
  }
  if (rank != 0 || file != 8) return false;
  while (*s == ' ') ++s;
  if (*s == 'w' || *s == 'b') B.stm = (*s++ == 'b');
  else if (*s) return false;
  if (popcnt(B.byType[KING] & B.byColor[WHITE]) != 1 || popcnt(B.byType[KING] & B.byColor[BLACK]) != 1)
    return false;
  if (popcnt(B.byType[0]) > 32 || (B.byType[PAWN] & 0xFF000000000000FFull)) return false;
  while (*s == ' ') ++s;
  while (*s && *s != ' ') {
    char t = *s++;
    if (t == '-') continue;
    int c = islower((unsigned char)t) ? BLACK : WHITE;
    char u = (char)toupper((unsigned char)t);
    int base = c == WHITE ? 0 : 56, rsq = -1;
    Bitboard rooks = B.byType[ROOK] & color_bb(B, c) & (0xFFull << base);
    if (u == 'K') {
      if (rooks) rsq = 63 - __builtin_clzll(rooks);
    } else if (u == 'Q') {
      if (rooks) rsq = lsb(rooks);
    } else if (u >= 'A' && u <= 'H')
      rsq = base + (u - 'A');
    else
      continue;
    int ksq = king_square(B, c);
    if (rsq < 0 || !(rooks & sqbb(rsq)) || (ksq >> 3) != (base >> 3)) continue;
    B.castle_rook[2 * c + (rsq > ksq ? 0 : 1)] = (uint8_t)rsq;
  }
  while (*s == ' ') ++s;
  if (s[0] >= 'a' && s[0] <= 'h' && s[1] == (B.stm == WHITE ? '6' : '3')) {
    int ep = (s[1] - '1') * 8 + (s[0] - 'a');
    int us = B.stm, up = us == WHITE ? 8 : -8;
    bool ok = (T.pawn[us ^ 1][ep] & B.byType[PAWN] & color_bb(B, us)) != 0 &&
              (B.byType[PAWN] & color_bb(B, us ^ 1) & sqbb(ep - up)) != 0 &&
              !(B.byType[0] & (sqbb(ep) | sqbb(ep + up)));
    if (ok) B.ep = (uint8_t)ep;
  }
  while (*s && *s != ' ') ++s;
  while (*s == ' ') ++s;
  if (*s) {
    long r = strtol(s, nullptr, 10);
    B.rule50 = (uint16_t)(r < 0 ? 0 : r > 65535 ? 65535 : r);
    while (*s && *s != ' ') ++s;
    while (*s == ' ') ++s;
    if (*s) {
      long f = strtol(s, nullptr, 10);
      B.fullmove = (uint16_t)(f < 1 ? 1 : f > 65535 ? 65535 : f);
    }
  }
  int oksq = king_square(B, B.stm ^ 1);
  if (attackers_to(B, T, oksq, B.byType[0]) & color_bb(B, B.stm)) return false;
  return true;
}

inline int board_to_fen(const Board &B, char *out, size_t cap) {
  char buf[128];
  int k = 0;
  for (int r = 7; r >= 0; --r) {
    int empty = 0;
    for (int f = 0; f < 8; ++f) {
      int pc = piece_on(B, r * 8 + f);
      if (!pc) {
        ++empty;
        continue;
      }
      if (empty) buf[k++] = (char)('0' + empty), empty = 0;
      char c = "?PNBRQK?"[pc & 7];
      buf[k++] = (pc >> 3) ? (char)tolower(c) : c;
    }
    if (empty) buf[k++] = (char)('0' + empty);
    if (r) buf[k++] = '/';
  }
  buf[k++] = ' ';
  buf[k++] = B.stm ? 'b' : 'w';
  buf[k++] = ' ';
  bool any = false;
  for (int i = 0; i < 4; ++i) {
    int rsq = B.castle_rook[i];
    if (rsq == SQ_NONE) continue;
    int c = i >> 1;
    Bitboard rooks = B.byType[ROOK] & color_bb(B, c) & (0xFFull << (c ? 56 : 0));
    bool outer = (i & 1) == 0 ? !(rooks & ~((sqbb(rsq) << 1) - 1)) : !(rooks & (sqbb(rsq) - 1));
    char ch = outer ? ((i & 1) == 0 ? 'K' : 'Q') : (char)('A' + (rsq & 7));
    buf[k++] = c ? (char)tolower(ch) : ch;
    any = true;
  }
  if (!any) buf[k++] = '-';
  buf[k++] = ' ';
  if (B.ep != SQ_NONE) buf[k++] = (char)('a' + (B.ep & 7)), buf[k++] = (char)('1' + (B.ep >> 3));
  else buf[k++] = '-';
  k += snprintf(buf + k, sizeof(buf) - (size_t)k, " %d %d", B.rule50, B.fullmove);
  if ((size_t)k + 1 > cap) return -1;
  memcpy(out, buf, (size_t)k + 1);
  return k;
}

inline int legal_moves(const Board &B, uint16_t *mv) {
  int n = 0;
  gen_legal(B, host_tables(), [&](uint16_t m) { mv[n++] = m; });
  return n;
}

inline Board random_playout(uint64_t seed, int max_plies) { return random_playout(seed, max_plies, host_tables()); }

} // namespace gn
