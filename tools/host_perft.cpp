// Host build of the product chess core (fishnet_amd/csrc/chess.h) for CPU
// debugging: prints perft divide for a FEN.  hipcc compiles it as host code.
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../fishnet_amd/csrc/host_board.h"
namespace gn {
const Tables &host_tables() {
  static Tables T = [] { Tables t; init_tables(t); return t; }();
  return T;
}
}
using namespace gn;
static uint64_t perft(const Board &B, int d) {
  uint16_t mv[256];
  int n = legal_moves(B, mv);
  if (d <= 1) return n;
  uint64_t s = 0;
  for (int i = 0; i < n; ++i) s += perft(do_move(B, mv[i]), d - 1);
  return s;
}
extern "C" uint64_t bfs_perft(const char *fen, int depth);
extern "C" int find_pack_bug(const gn::Board &B, int d);
int main(int argc, char **argv) {
  if (argc > 4) { Board B0; parse_fen(argv[1], B0); return find_pack_bug(B0, atoi(argv[2])); }
  if (argc > 3) { printf("bfs %llu\n", (unsigned long long)bfs_perft(argv[1], atoi(argv[2]))); return 0; }
  Board B;
  if (!parse_fen(argv[1], B)) { printf("bad fen\n"); return 1; }
  int d = atoi(argv[2]);
  uint16_t mv[256];
  int n = legal_moves(B, mv);
  uint64_t tot = 0;
  for (int i = 0; i < n; ++i) {
    Board C = do_move(B, mv[i]);
    uint64_t c = d > 1 ? perft(C, d - 1) : 1;
    char fen[128]; board_to_fen(C, fen, sizeof fen);
    int m = mv[i], f = (m >> 6) & 63, t = m & 63;
    printf("%c%d%c%d %llu %s\n", 'a' + (f & 7), 1 + (f >> 3), 'a' + (t & 7), 1 + (t >> 3), (unsigned long long)c, fen);
    tot += c;
  }
  printf("total %llu\n", (unsigned long long)tot);
}
// (appended) BFS through the packed format, like the device path
extern "C" uint64_t bfs_perft(const char *fen, int depth) {
  Board B; parse_fen(fen, B);
  std::vector<gn_board> cur(1), nxt;
  pack(B, cur[0]);
  for (int l = 1; l < depth; ++l) {
    nxt.clear();
    for (auto &p : cur) { Board X; if (!unpack(p, X)) continue; gen_legal(X, host_tables(), [&](uint16_t m) { gn_board q; pack(do_move(X, m), q); nxt.push_back(q); }); }
    cur.swap(nxt);
  }
  uint64_t s = 0;
  for (auto &p : cur) { Board X; if (unpack(p, X)) gen_legal(X, host_tables(), [&](uint16_t) { ++s; }); }
  return s;
}
extern "C" int find_pack_bug(const Board &B, int d) {
  uint16_t mv[256], mv2[256];
  gn_board p; pack(B, p); Board X; bool ok = unpack(p, X);
  int n = legal_moves(B, mv), n2 = ok ? legal_moves(X, mv2) : -1;
  if (n != n2) {
    char f1[128], f2[128]; board_to_fen(B, f1, 128); if (ok) board_to_fen(X, f2, 128); else f2[0]=0;
    printf("MISMATCH %d vs %d\n  %s\n  %s ok=%d castle=%x\n", n, n2, f1, f2, ok, p.castle);
    for (int i=0;i<4;++i) printf("  B.cr[%d]=%d X.cr[%d]=%d\n", i, B.castle_rook[i], i, X.castle_rook[i]);
    return 1;
  }
  if (d <= 1) return 0;
  for (int i = 0; i < n; ++i) if (find_pack_bug(do_move(B, mv[i]), d - 1)) return 1;
  return 0;
}
