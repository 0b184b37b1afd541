/*
 * oracle.h — CPU restatement of the gpu_nnue hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  It is the checker, never the thing shipped or measured as the
 * product.  The product path (fishnet_amd/, libgpu_nnue.so) must not link it.
 *
 * What it restates (the reference's own engine code is NOT in /root/reference:
 * the `Stockfish/` submodule of ounben/fishnet is empty, .gitmodules:1-3):
 *   - Stockfish 17.1-era NNUE evaluation (network file format, HalfKAv2_hm
 *     features, feature transformer, layer stack, Eval::evaluate epilogue),
 *     restated from the published algorithm;
 *   - legal move generation + perft, written as a
 *     simple mailbox generator independent of the product's bitboard code.
 *
 * Parity status: perft is PINNED by public known-answer tables
 * (tests/golden/perft.json).  The NNUE arithmetic is "parity unpinned": no
 * Stockfish source, binary or .nnue net exists in this container, so the
 * restatement is checked only against self-consistency goldens
 * (tests/golden/eval_*.json) and hand-derived unit cases.
 */
#ifndef FISHNET_ORACLE_H
#define FISHNET_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* evaluation modes (mirror of include/gpu_nnue.h GN_MODE_*) */
#define OR_MODE_FULL 0  /* Eval::evaluate: small/big selection + big re-eval */
#define OR_MODE_BIG 1   /* big net only, epilogue with smallNet = false      */
#define OR_MODE_SMALL 2 /* small net only, epilogue with smallNet = true     */

/* result flags (mirror of GN_FLAG_*) */
#define OR_FLAG_IN_CHECK 1u
#define OR_FLAG_SMALLNET 2u
#define OR_FLAG_BAD_FEN 4u
#define OR_FLAG_REEVAL 8u
#define OR_FLAG_MATE 32u     /* score is a mate distance                            */
#define OR_FLAG_NO_SCORE 64u /* no score (bad FEN, or a child record)               */
#define OR_FLAG_SEARCHED 128u /* score from the in-check rule, best_move set        */
#define OR_FLAG_NO_MOVES 256u /* no legal move (checkmate / stalemate)              */

/* Mirror of gn_eval (ABI v3).  score: the score fishnet posts, by the rule gpu_nnue.h
 * states at gn_eval (restated in or_score below from that text and from what the
 * reference requires: a `score cp|mate` for every analysed position,
 * /root/reference/src/stockfish.rs:366-368, src/ipc.rs:56). */
typedef struct {
  int32_t psqt;       /* NetworkOutput.psqt of the net that produced final  */
  int32_t positional; /* NetworkOutput.positional of that net               */
  int32_t final_v;    /* Eval::evaluate(optimism = 0), side-to-move POV     */
  int32_t final_cp;   /* UCIEngine::to_cp(final_v): the printed centipawns  */
  int32_t score;      /* cp, or moves to mate with OR_FLAG_MATE              */
  uint16_t flags;
  uint16_t best_move; /* the in-check rule's reply (Stockfish encoding)     */
} or_eval;

typedef struct or_net or_net;

/* Load a .nnue file (Stockfish format).  Returns 0 on success, negative on error
 * (message written to err). */
int or_net_load(const char *path, or_net **out, char *err, int errlen);
int or_net_load_mem(const uint8_t *buf, size_t len, or_net **out, char *err, int errlen);
void or_net_free(or_net *net);
int or_net_l1(const or_net *net);
uint32_t or_net_hash(const or_net *net);
/* expected network hash for a given L1 width (FT hash ^ architecture hash) */
uint32_t or_expected_hash(int l1, uint32_t *ft_hash, uint32_t *arch_hash);

/* evaluate one FEN (a position: the score rule applies).  big or small may be NULL when
 * the mode does not need it. */
int or_eval_fen(const or_net *big, const or_net *small, const char *fen, int mode, or_eval *out);
/* evaluate a batch with `threads` POSIX threads (threads <= 0: 1) */
int or_eval_fens(const or_net *big, const or_net *small, const char *const *fens, size_t n,
                 int mode, or_eval *out, int threads);

/* network building blocks, exposed for unit tests */
int or_features(const char *fen, int perspective, uint32_t *idx, int cap);
int or_accumulate(const or_net *net, const char *fen, int perspective, int16_t *acc, int32_t *psqt8);
int or_net_output(const or_net *net, const char *fen, int32_t *psqt, int32_t *positional);

/* move generation.  Moves use Stockfish's 16-bit encoding:
 * to | from << 6 | (promo_type - KNIGHT) << 12 | type << 14, type 1 = promotion,
 * 2 = en passant, 3 = castling (to = rook square). */
int or_legal_moves(const char *fen, uint16_t *moves, int cap);
int or_child_fen(const char *fen, uint16_t move, char *out, int cap);
int or_normalize_fen(const char *fen, char *out, int cap);
uint64_t or_perft(const char *fen, int depth); /* UINT64_MAX on a bad FEN */

/* parent + every legal child evaluated (children in Stockfish movegen order is
 * NOT promised; moves[] reports the order used).  The parent is a position (scored),
 * the children are child records (OR_FLAG_NO_SCORE).  Returns the child count, or
 * negative on error / cap overflow. */
int or_expand_eval(const or_net *big, const or_net *small, const char *fen, int mode,
                   or_eval *parent, uint16_t *moves, or_eval *children, int cap);

/* or_expand_eval with the children's accumulators updated incrementally from the
 * parent's (a king move refreshes that perspective), as Stockfish does on the CPU. */
int or_expand_eval_inc(const or_net *big, const or_net *small, const char *fen, int mode,
                       or_eval *parent, uint16_t *moves, or_eval *children, int cap);
/* n parents expanded by `threads` POSIX threads (work-stealing in chunks of 16):
 * parents[i], child_counts[i] (negative: bad FEN), children[256 * i + k] when
 * children is not NULL.  incremental selects or_expand_eval_inc / or_expand_eval. */
int or_expand_eval_batch(const or_net *big, const or_net *small, const char *const *fens, size_t n, int mode,
                         int incremental, int threads, or_eval *parents, int32_t *child_counts, or_eval *children);

#ifdef __cplusplus
}
#endif
#endif
