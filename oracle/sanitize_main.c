/*
 * sanitize_main.c — drives the oracle under AddressSanitizer + UBSan (TEST INFRASTRUCTURE
 * ONLY: built by `make -C oracle sanitize`, run by tests/test_oracle.py::
 * test_oracle_under_sanitizers).  A separate executable, so the sanitizer runtime is the
 * program's own (no preload into Python).
 *
 * usage: oracle_sanitize <big.nnue> <small.nnue> <fens.txt>
 * For every FEN line: or_eval_fen in the three modes, or_expand_eval and
 * or_expand_eval_inc (BIG mode; their results must agree), and perft(2).  Prints one
 * line per FEN: "<final_v FULL> <final_cp FULL> <n children> <sum of child final_v> <perft2>",
 * or "bad" for a rejected FEN.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

int main(int argc, char **argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: %s big.nnue small.nnue fens.txt\n", argv[0]);
    return 2;
  }
  char err[256];
  or_net *big = NULL, *small = NULL;
  if (or_net_load(argv[1], &big, err, sizeof err) || or_net_load(argv[2], &small, err, sizeof err)) {
    fprintf(stderr, "net: %s\n", err);
    return 2;
  }
  FILE *f = fopen(argv[3], "r");
  if (!f) return 2;
  char line[512];
  or_eval par, par2, *ch = malloc(256 * sizeof(or_eval)), *ch2 = malloc(256 * sizeof(or_eval));
  uint16_t mv[256], mv2[256];
  int rc = 0;
  while (fgets(line, sizeof line, f)) {
    line[strcspn(line, "\r\n")] = 0;
    if (!line[0]) continue;
    or_eval e[3];
    int bad = 0;
    for (int m = 0; m < 3; ++m) bad |= or_eval_fen(big, small, line, m, &e[m]) != 0;
    if (bad) {
      printf("bad\n");
      continue;
    }
    const int n = or_expand_eval(big, small, line, OR_MODE_BIG, &par, mv, ch, 256);
    const int n2 = or_expand_eval_inc(big, small, line, OR_MODE_BIG, &par2, mv2, ch2, 256);
    if (n != n2 || n < 0 || memcmp(&par, &par2, sizeof par) || memcmp(mv, mv2, (size_t)(n > 0 ? n : 0) * 2) ||
        memcmp(ch, ch2, (size_t)(n > 0 ? n : 0) * sizeof(or_eval))) {
      fprintf(stderr, "refresh and incremental expansion differ: %s\n", line);
      rc = 1;
    }
    long long sum = 0;
    for (int k = 0; k < n; ++k) sum += ch[k].final_v;
    printf("%d %d %d %lld %llu\n", e[0].final_v, e[0].final_cp, n, sum, (unsigned long long)or_perft(line, 2));
  }
  fclose(f);
  free(ch), free(ch2);
  or_net_free(big), or_net_free(small);
  return rc;
}
