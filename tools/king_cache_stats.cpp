// Host count of king-move refresh rows with and without a per-game king cache
// (DESIGN.md §4 step 6), on random 80-ply games like the bench's (host order of moves).
// Build: hipcc -O2 -std=c++17 tools/king_cache_stats.cpp -o /tmp/king_cache_stats
#include <stdio.h>
#include <stdlib.h>
#include <map>
#include "../fishnet_amd/csrc/host_board.h"
namespace gn {
const Tables &host_tables() { static Tables T = [] { Tables t; init_tables(t); return t; }(); return T; }
}
using namespace gn;
int main(int argc, char **argv) {
  const Tables &T = host_tables();
  int games = argc > 1 ? atoi(argv[1]) : 2000, plies = 80;
  unsigned long long par_rows = 0, delta_rows = 0, king_rows = 0, king_children = 0, children = 0, finny_rows = 0, finny_hits = 0;
  for (int g = 0; g < games; ++g) {
    Xoshiro rng(0x5EED0000ull + g);
    Board B = start_position();
    std::map<int, Board> cache; // key (persp*64 + kt) -> child board
    for (int k = 0; k <= plies; ++k) {
      uint16_t mv[256];
      int n = legal_moves(B, mv);
      int P = __builtin_popcountll(B.byType[0]);
      par_rows += 2 * (P + 1);
      for (int i = 0; i < n; ++i) {
        Dirty d; Board C = do_move(B, mv[i], &d);
        ++children;
        if (d.king_moved) {
          ++king_children;
          int Pc = __builtin_popcountll(C.byType[0]);
          king_rows += Pc + 1 + d.n_rem + d.n_add;
          int h = B.stm, kt = king_square(C, h), key = h * 64 + kt;
          auto it = cache.find(key);
          int diff = 1 << 30;
          if (it != cache.end()) {
            diff = 0;
            for (int s = 0; s < 64; ++s) if (piece_on(it->second, s) != piece_on(C, s)) ++diff;
          }
          if (diff + 1 < Pc + 1) { finny_rows += diff + 1; ++finny_hits; } else finny_rows += Pc + 1;
          finny_rows += d.n_rem + d.n_add;
          cache[key] = C;
        } else delta_rows += 2 * (d.n_rem + d.n_add);
      }
      if (n && B.rule50 < 100) B = do_move(B, mv[rng.below((uint32_t)n)] , nullptr); // NOTE: order may differ from nth_legal
    }
  }
  printf("children %llu king_children %llu (%.1f%%)\nrows: parents %llu deltas %llu king %llu ; finny king %llu (hits %llu)\n",
         children, king_children, 100.0 * king_children / children, par_rows, delta_rows, king_rows, finny_rows, finny_hits);
}
