/*
 * gpu_nnue.h — C-ABI of libgpu_nnue.so, the MI355X (gfx950) batched Stockfish
 * NNUE evaluator for fishnet.
 *
 * Boundary being replaced / extended (reference = ounben/fishnet @ 2025-05-09):
 *   - StockfishStub::go_multiple(Chunk) -> Result<Vec<PositionResponse>, ChunkFailed>
 *     /root/reference/src/stockfish.rs:36-47 — the engine plugin API.  A GPU
 *     backend sits beside it; the Rust `gpu_nnue` module calls
 *     the functions below from tokio::task::spawn_blocking.
 *   - The static evaluation those engine processes run at every search leaf
 *     (Stockfish `Eval::evaluate`, inside the empty Stockfish submodule,
 *     /root/reference/.gitmodules:1-3) is what gn_evaluate_batch computes.
 *   - Nets: the reference ships nn-1c0000000000.nnue (big) and
 *     nn-37f18f62d772.nnue (small) next to the engine (/root/reference/build.rs:8-9,
 *     src/assets.rs:186-226); gn_load_net takes those files.
 *
 * Conventions: plain pointers and sizes; the caller owns every input and output
 * buffer, the library owns device memory.  Every function returns GN_OK (0) or a
 * negative GN_E_* code and never aborts or throws across the ABI; the message of
 * the last failure on the calling thread is gn_last_error().  A gn_ctx may be
 * shared between threads: calls on one context are serialised internally.
 */
#ifndef GPU_NNUE_H
#define GPU_NNUE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* v2: gn_eval carries final_cp (UCIEngine::to_cp) and 16-bit flags; gn_eval_params
 * carries the win-rate model; expansion shards over every device of the context.
 * v3: gn_eval is 24 bytes: final_cp is int32 and every evaluated position carries the
 * score fishnet posts (score, GN_FLAG_MATE / GN_FLAG_SEARCHED / GN_FLAG_NO_MOVES,
 * best_move): checkmate, stalemate and in-check positions included. */
/* v4: the host-buffer expansion calls (gn_expand_and_evaluate, gn_evaluate_games with
 * children) return every legal child as a 12-byte gn_child (psqt, positional, final_cp + flags:
 * the north star's (i32 psqt, i32 positional, i32 final_cp)) instead of a 24-byte gn_eval;
 * GN_OPT_CHUNK_PARENTS; GN_STAT_CHAIN_FALLBACKS removed (the planned expansion has no
 * fallback); the device-resident calls are documented as blocking (they were since v3). */
#define GN_ABI_VERSION 4

#if defined(__GNUC__)
#define GN_API __attribute__((visibility("default")))
#else
#define GN_API
#endif

/* return codes */
#define GN_OK 0
#define GN_E_INVALID (-1)  /* bad argument                                    */
#define GN_E_IO (-2)       /* cannot read a net file                          */
#define GN_E_FORMAT (-3)   /* not a supported .nnue (version/hash/size)       */
#define GN_E_HIP (-4)      /* HIP runtime error (message has the detail)      */
#define GN_E_NOMEM (-5)    /* host or device allocation failed                */
#define GN_E_CAPACITY (-6) /* caller's output buffer too small                */
#define GN_E_NODEVICE (-7) /* no usable gfx950 device                         */
#define GN_E_NONET (-8)    /* the requested mode needs a net that is not loaded */
#define GN_E_ILLEGAL_MOVE (-9) /* a game's UCI move does not resolve to a legal move */

/* evaluation modes */
#define GN_MODE_FULL 0  /* Eval::evaluate: small net when |simple_eval| > 962,
                           big-net re-evaluation when |nnue| < 236            */
#define GN_MODE_BIG 1   /* big net for every position (epilogue: smallNet=false) */
#define GN_MODE_SMALL 2 /* small net for every position (epilogue: smallNet=true) */

/* options (gn_set_option / gn_get_option) */
#define GN_OPT_CHUNK_PARENTS 6        /* host-buffer expansion pipeline (gn_expand_and_evaluate,
                                         gn_evaluate_games with children): parents per chunk,
                                         cut at game starts; 0 (default): automatic (whole
                                         games, >= 165,888 parents per chunk, a short last
                                         chunk).  Results are identical for every value.   */
#define GN_OPT_COALESCE 7             /* 1 (default): concurrent gn_evaluate_batch calls on one
                                         context are merged into one launch (each call
                                         queues; one call leads a launch over every queued
                                         call of its mode; a lone call runs at once, no
                                         timer); 0: calls run one after another.  Results
                                         are identical either way.                        */
#define GN_OPT_FAST_BATCH 9           /* 1 (default): a gn_evaluate_batch of <= 4,096 positions on
                                         a one-device context runs as one captured HIP graph
                                         (upload, evaluation, both levels of the score rule's
                                         in-check replies, download: one host synchronisation
                                         per call); 0: the general path (a launch sequence with
                                         a host round trip per reply level).  Results are
                                         identical either way.                              */
#define GN_OPT_EXPAND_PIPELINE 10     /* 1: consecutive planned expansions of one call
                                         (gn_time_expand_device's iterations, the host-buffer
                                         pipeline's chunks) overlap: expansion k + 1's child
                                         generation and plan run on a second stream while
                                         expansion k's finalize and score rule run (two
                                         buffer sets); 2 (default): the next child
                                         generation and plan start while expansion k's row
                                         stream still runs (151.3 against 153.9 ms per bench
                                         step unpipelined); 0: one after another.  Results
                                         are identical for every value.                     */
#define GN_OPT_INCREMENTAL_CHILDREN 1 /* 1 (default): children from the parent accumulators
                                         by add/sub deltas; 0: full refresh per child    */
#define GN_OPT_XCD_SWIZZLE 2          /* bit mask, default 9: each XCD takes a contiguous
                                         range of parents (bit 0, small-net expansion) / of
                                         16-position tiles (bit 1, batch evaluation) / of
                                         blocks (bit 2, big-net expansion); 0: dispatch order
                                         (big-net expansion: blocks claimed in order by an
                                         atomic counter); bit 3 (big-net expansion, without
                                         bit 2; default): each XCD claims blocks of its own
                                         eighth of the order, then of the others' (stream
                                         205.1 -> 203.6 ms against one counter)          */
#define GN_OPT_KING_SORT 3            /* 1 (default): evaluate a batch of >= 1,024 positions
                                         (2: of any size) in (white king, black
                                         king) square order for L2 / Infinity-Cache
                                         locality, then (big net) by layer-stack bucket and
                                         30 home-square bits (ranks 1, 2, 7, 8 without
                                         e1/e8: the start position's piece still stands
                                         there) so that 16-position tiles share rows
                                         gathered once per tile and one layer stack; small
                                         net: by bucket, then kings; results in input
                                         order; 0: input order                            */
#define GN_OPT_KING_CACHE 5           /* 1 (default): with the chained walk, a king-move
                                         child's refresh starts from the accumulator the
                                         workgroup last computed for that (perspective,
                                         king square) in the same block, plus the placement
                                         difference, when that is shorter (Stockfish's
                                         AccumulatorCaches analog); 0: full refresh.
                                         Results are identical either way.               */
#define GN_OPT_CHAIN 4                /* expansion (big net): a workgroup walks blocks of up to
                                         this many consecutive parents (default 81: one
                                         80-ply game); a parent that is a child of the
                                         previous one (same placement) starts from that
                                         child's accumulators instead of a refresh.
                                         Shortened when the blocks would not fill the GPU;
                                         -k: exactly k.  0, 1 or -1: every parent
                                         refreshes.  Results are identical either way.    */
#define GN_OPT_STREAM_SLICES 8        /* expansion with a 3072-wide big net: 3 (default): the
                                         accumulator columns in three slices of 1,024, one
                                         stream launch each over every entry, so that an
                                         XCD's L2 holds the slice's rows of the king buckets
                                         in flight; 1: one launch over whole rows.  Results
                                         are identical either way.  The slices' fc_0 partial
                                         sums take 200 B of device memory per evaluated
                                         position (parents + children of a call or chunk);
                                         when that allocation fails the call runs the
                                         whole-row stream instead.                        */

/* read-only statistics (gn_get_option) */
#define GN_STAT_PLAN_NS 101           /* the last gn_time_expand_device's planned big net
                                         (max over devices, per iteration, nanoseconds):
                                         plan_kernel (lists, tiles, PSQT) ...            */
#define GN_STAT_STREAM_NS 102         /* ... and stream_eval_kernel (row stream + layer
                                         stack; all its launches: three column slices by
                                         default), the expansion's dominant kernel ...   */
#define GN_STAT_FINISH_NS 104         /* ... and the column-sliced stream's layer-stack
                                         finish (slice_finish_kernel; ~0 by default, where
                                         finalize computes each output itself, and with
                                         one launch)                                       */
#define GN_STAT_SCRATCH_PADS 103      /* no-op entries the last planned expansion inserted
                                         (per device, summed) so that every king-cache load
                                         sits >= ring depth (4) list entries after the
                                         list's last king-cache store (the load then issues
                                         after the store, from the same lanes)            */
/* stage times of the last gn_evaluate_games / gn_expand_and_evaluate (nanoseconds; per-device
 * stages: the slowest device).  The expansion runs in chunks of whole games; a drain thread
 * downloads chunk c's records on a copy stream while chunk c + 1 computes.               */
#define GN_STAT_HOST_PARSE_NS 110     /* host: root FENs / FENs parsed, UCI moves tokenized */
#define GN_STAT_HOST_UPLOAD_NS 111    /* host -> device copies of the inputs               */
#define GN_STAT_HOST_REPLAY_NS 112    /* the GPU replay of the games' moves (games only)   */
#define GN_STAT_HOST_COMPUTE_NS 113   /* children, evaluation and score rule, all chunks   */
#define GN_STAT_HOST_DOWNLOAD_NS 114  /* device -> host result copies, all chunks (they
                                         overlap the next chunk's compute)               */
#define GN_STAT_HOST_TAIL_NS 115      /* the downloads still running after the last chunk
                                         computed (not overlapped)                        */
#define GN_STAT_HOST_TOTAL_NS 116     /* the whole call                                    */
#define GN_STAT_BATCH_LAUNCHES 117    /* merged gn_evaluate_batch launches since load ...   */
#define GN_STAT_BATCH_CALLS 118       /* ... and the calls they served (GN_OPT_COALESCE)    */
#define GN_STAT_FAST_BATCHES 119      /* evaluations run by the captured small-batch graphs
                                         (GN_OPT_FAST_BATCH) since load ...                 */
#define GN_STAT_FAST_FALLBACKS 120    /* ... and those rerun on the general path because a
                                         reply level exceeded the graph's capacity          */

/* per-position flags */
#define GN_FLAG_IN_CHECK 1u /* side to move in check: Stockfish has no static eval
                               (Eval::evaluate asserts !checkers); values are still
                               computed but are not a Stockfish result            */
#define GN_FLAG_SMALLNET 2u /* final_v came from the small net                    */
#define GN_FLAG_BAD_FEN 4u  /* unparsable / unsupported position; values are 0     */
#define GN_FLAG_REEVAL 8u   /* small net was run, then the big net re-evaluated   */
#define GN_FLAG_SKIPPED 16u /* listed in skipPositions: not evaluated, values 0    */
#define GN_FLAG_MATE 32u    /* score is a mate distance (UCI `score mate <score>`)  */
#define GN_FLAG_NO_SCORE 64u /* no score: skipped / bad position, or a child record */
#define GN_FLAG_SEARCHED 128u /* score from the in-check rule over the legal replies
                                 (best_move set), not from the static evaluation   */
#define GN_FLAG_NO_MOVES 256u /* no legal move: checkmate (with IN_CHECK) or stalemate */

/* One result.  psqt/positional are Network::evaluate's NetworkOutput (already
 * divided by OutputScale = 16) of the net that produced final_v; final_v is
 * Eval::evaluate(pos, optimism = 0) in internal Value units; final_cp is
 * final_v in centipawns as Stockfish prints it (UCIEngine::to_cp: the win-rate
 * model's a(material), round(100 * v / a)); all side-to-move POV.
 *
 * score is what fishnet posts for the position: the `score cp X` / `score mate N` a
 * Stockfish `go` prints and stockfish.rs:419-431 parses; fishnet requires one for
 * every analysed position (stockfish.rs:366-368, ipc.rs:56 `expect("got score")`).
 * The rule, for every position a call is given (batch, game and parent positions):
 *   - no legal move: checkmate -> `mate 0` (GN_FLAG_MATE, score 0), stalemate -> `cp 0`
 *     (what Stockfish prints at depth 0); GN_FLAG_NO_MOVES;
 *   - not in check: score = final_cp (the static evaluation);
 *   - in check with legal moves (Stockfish has no static eval there): a check extension,
 *     value(p, d) = max over legal replies c of -value(c, d - 1) from d = 2, where a reply
 *     with no legal move is mated (-VALUE_MATE = -32000) or stalemated (0), a reply not in
 *     check -- or any reply at d = 0 -- takes its static final_v, and mate values move one
 *     ply toward zero per level (VALUE_MATE - ply); ties go to the smaller move encoding.
 *     score = `mate (ply + 1) / 2` / `mate -ply / 2` for |value| >= 31754
 *     (VALUE_MATE_IN_MAX_PLY), else to_cp(value) with this position's material;
 *     GN_FLAG_SEARCHED, best_move = the reply (Stockfish encoding).
 * Child and grandchild records of the expansion calls carry GN_FLAG_NO_SCORE (score 0):
 * they are search data, not positions fishnet posts. */
typedef struct gn_eval {
  int32_t psqt;
  int32_t positional;
  int32_t final_v;
  int32_t final_cp;
  int32_t score;
  uint16_t flags;
  uint16_t best_move;
} gn_eval;

/* One legal child as the host-buffer expansion calls return it (ABI v4, 12 bytes): the child's
 * static evaluation, north star `(i32 psqt, i32 positional, i32 final_cp)`, with the flags
 * packed beside final_cp.  psqt / positional / final_cp are those of the child's gn_eval record
 * (side-to-move POV); cp_flags = (final_cp & 0xFFFFFF) | (flags & 0xFF) << 24: final_cp as a
 * signed 24-bit integer (|final_cp| < 2^23 always: gn_set_eval_params keeps the win-rate
 * model's a(material) >= 1, and |final_v| <= value_clamp), flags the record's low 8 flag bits
 * (GN_FLAG_IN_CHECK, GN_FLAG_SMALLNET, GN_FLAG_REEVAL; GN_FLAG_NO_SCORE is always set: a child
 * carries no score).  Decode with GN_CHILD_FINAL_CP / GN_CHILD_FLAGS. */
typedef struct gn_child {
  int32_t psqt;
  int32_t positional;
  int32_t cp_flags;
} gn_child;
#define GN_CHILD_FINAL_CP(c) ((int32_t)((uint32_t)(c).cp_flags << 8) >> 8)
#define GN_CHILD_FLAGS(c) ((uint32_t)(c).cp_flags >> 24)

/* Packed position, 32 bytes, the device input format.
 *   occ      occupied squares (bit s = square s, a1 = 0 .. h8 = 63)
 *   pc       piece codes (Stockfish encoding: 1..6 white P N B R Q K, 9..14 black)
 *            of the occupied squares in ascending square order, two per byte,
 *            low nibble first
 *   stm_ep   bit 7 = side to move (1 = black); bits 0..6 = en-passant square
 *            or 64 when none
 *   castle   4 nibbles [white O-O, white O-O-O, black O-O, black O-O-O]:
 *            bit 3 = right present, bits 0..2 = file of the castling rook
 *   rule50   half-move clock; fullmove = full-move number                    */
typedef struct gn_board {
  uint64_t occ;
  uint8_t pc[16];
  uint8_t stm_ep;
  uint8_t reserved;
  uint16_t castle;
  uint16_t rule50;
  uint16_t fullmove;
} gn_board;

/* Eval::evaluate constants (defaults = Stockfish 17.1). */
typedef struct gn_eval_params {
  int32_t small_net_threshold; /* 962   |simple_eval| above which the small net is used */
  int32_t psqt_weight;         /* 125   nnue = (psqt_w*psqt + pos_w*positional) / 128  */
  int32_t positional_weight;   /* 131                                                */
  int32_t reeval_threshold;    /* 236   small-net |nnue| below which big re-evaluates */
  int32_t complexity_div_small;/* 18000 nnue -= nnue * |psqt - positional| / div      */
  int32_t complexity_div_big;  /* 18000                                              */
  int32_t material_pawn_small; /* 535   material = k * pawns + non_pawn_material     */
  int32_t material_pawn_big;   /* 535                                                */
  int32_t material_base;       /* 77777 v = nnue * (base + material) / base          */
  int32_t rule50_div;          /* 212   v -= v * rule50 / div                        */
  int32_t value_clamp;         /* 31506 |v| <= VALUE_TB_WIN_IN_MAX_PLY - 1           */
  int32_t piece_value[5];      /* 208 781 825 1276 2538 (P N B R Q)                  */
  /* UCIEngine::to_cp / win_rate_params (Stockfish 17-era uci.cpp; recalled, parity
   * unpinned like the constants above):
   *   material = sum wdl_piece_weight[pt] * count(pt) over both colours (P N B R Q)
   *   m = clamp(material, wdl_material_min, wdl_material_max) / (double)wdl_material_anchor
   *   a = ((wdl_a[0] * m + wdl_a[1]) * m + wdl_a[2]) * m + wdl_a[3]   (no FMA contraction)
   *   final_cp = round(100 * final_v / a)                             (half away from zero) */
  double wdl_a[4];             /* -37.45051876 121.19101539 -132.78783573 420.70576692 */
  int32_t wdl_material_min;    /* 17 */
  int32_t wdl_material_max;    /* 78 */
  int32_t wdl_material_anchor; /* 58 */
  int32_t wdl_piece_weight[5]; /* 1 3 3 5 9 */
} gn_eval_params;

typedef struct gn_ctx gn_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
/* Load nets and upload them to each listed device (devices = NULL: device 0).
 * small_path may be NULL (then only GN_MODE_BIG works); big_path may be NULL
 * (then only GN_MODE_SMALL works). */
GN_API int gn_load_net(const char *big_path, const char *small_path, const int *devices, int n_devices,
                gn_ctx **out);
/* A file named like Stockfish's nets, "nn-" + 12 lowercase hex digits + ".nnue"
 * (build.rs:8-9), must hash to its name: the first 12 hex digits of its SHA-256
 * (the check Stockfish's `make net` does after download, build.rs:318-333);
 * otherwise gn_load_net fails with GN_E_FORMAT.  Other file names are not checked. */
/* Same from in-memory .nnue images (e.g. after an RCCL broadcast). */
GN_API int gn_load_net_memory(const uint8_t *big, size_t big_len, const uint8_t *small, size_t small_len,
                       const int *devices, int n_devices, gn_ctx **out);
/* Nets from fishnet's asset archive (assets.ar.zst: a zstd-compressed `ar` archive, as
 * /root/reference/build.rs:398-420 writes it and src/assets.rs:186-226 reads it; a plain
 * `ar` works too).  big_member / small_member: member names (e.g. "nn-1c0000000000.nnue"),
 * or NULL for the first .nnue member of that kind (big: L1 3072 / 1024; small: 128).
 * Members named nn-<hex>.nnue are checked against their SHA-256 prefix.  zstd is
 * decoded by the system's libzstd.so.1, opened at run time. */
GN_API int gn_load_net_archive(const char *archive_path, const char *big_member, const char *small_member,
                               const int *devices, int n_devices, gn_ctx **out);
/* One member's bytes (CPU only): GN_E_CAPACITY with *size set when cap is too small. */
GN_API int gn_archive_read(const char *archive_path, const char *member, uint8_t *buf, size_t cap, size_t *size);
GN_API void gn_free(gn_ctx *ctx);
GN_API const char *gn_last_error(void); /* thread-local; valid until the next call */
GN_API int gn_abi_version(void);
GN_API int gn_get_eval_params(const gn_ctx *ctx, gn_eval_params *out);
GN_API int gn_set_eval_params(gn_ctx *ctx, const gn_eval_params *params);
GN_API int gn_set_option(gn_ctx *ctx, int option, int64_t value);
GN_API int gn_get_option(const gn_ctx *ctx, int option, int64_t *value);
/* SHA-256 of a buffer as 64 lowercase hex digits + NUL (net provenance; host only). */
GN_API int gn_net_sha256(const uint8_t *data, size_t len, char *hex65);
/* network hashes / widths actually loaded (0 when absent) */
GN_API int gn_net_info(const gn_ctx *ctx, int *big_l1, uint32_t *big_hash, int *small_l1, uint32_t *small_hash);

/* ---- host-buffer API (what the Rust gpu_nnue module calls) -------------- */
/* Evaluate n FENs (Chess960 castling accepted: KQkq, Shredder and X-FEN).
 * gn_evaluate_batch == gn_evaluate_batch_mode(..., GN_MODE_FULL, ...).
 * Bad FENs do not fail the batch: their entry carries GN_FLAG_BAD_FEN. */
GN_API int gn_evaluate_batch(gn_ctx *ctx, const char *const *fens, size_t n, gn_eval *out);
GN_API int gn_evaluate_batch_mode(gn_ctx *ctx, const char *const *fens, size_t n, int mode, gn_eval *out);

/* Every parent plus every legal child of it, sharded over every device of the
 * context (gn_partition, one host thread per device).  child_offsets[n+1] receives the
 * prefix sums (children of parent i are [child_offsets[i], child_offsets[i+1])),
 * child_moves / child_out receive one entry per child in the order the device
 * generator emits them (moves in Stockfish 16-bit encoding; castling = king
 * takes own rook; records as gn_child).  GN_E_CAPACITY when the children exceed cap
 * (child_offsets is still filled so the caller can retry with the right size). */
GN_API int gn_expand_and_evaluate(gn_ctx *ctx, const char *const *parent_fens, size_t n, int mode,
                           gn_eval *parent_out, uint32_t *child_offsets, uint16_t *child_moves,
                           gn_child *child_out, size_t cap);

/* ---- lichess analysis batches ------------------------------------------ */
/* One acquired batch as the server sends it (AcquireResponseBody,
 * /root/reference/src/api.rs:306-321): the root FEN, the game's UCI moves as
 * one whitespace-separated string (the wire form; NULL or "" = no moves) and
 * skipPositions (indices into positions 0..=moves). */
typedef struct gn_game {
  const char *root_fen;
  const char *uci_moves;
  const uint32_t *skip_positions;
  size_t n_skip;
} gn_game;

/* Replaces IncomingBatch::from_acquired (/root/reference/src/queue.rs:548-700)
 * for the evaluator: position i = root after i moves, i = 0..=moves.  Moves are
 * resolved as shakmaty 0.27.3's UciMove::to_move does (queue.rs:576): king onto
 * a castling rook = castling (Chess960 form), e1g1/e1c1-style king moves =
 * castling with the h/a rook (standard form), promotion letter n/b/r/q.  moves[]
 * receives them in Stockfish encoding (castling = king takes rook, i.e. the
 * Chess960 UCI the reference forwards, queue.rs:577).  A bad root FEN fails with
 * GN_E_INVALID, a move that is not legal with GN_E_ILLEGAL_MOVE (the reference
 * fails the whole batch, `uci.to_move(&pos)?`).  *n_positions = moves + 1 is set
 * on GN_E_CAPACITY too.  Host only, no context and no GPU needed. */
GN_API int gn_replay_game(const gn_game *game, gn_board *positions, uint8_t *skipped, uint16_t *moves, size_t cap,
                          size_t *n_positions);

/* Replay + evaluate n_games batches at once.  position_offsets[n_games + 1]:
 * positions of game g are [position_offsets[g], position_offsets[g + 1]);
 * game_status[g] = GN_OK or that game's GN_E_* (a failed game has no positions;
 * the other games are still evaluated and the call returns GN_OK).  Games are
 * sharded over the devices of the context, never split (gn_partition weighted by
 * evaluated positions), so a game's consecutive positions share a device.  Skipped
 * positions get GN_FLAG_SKIPPED and no children.  with_children != 0: also every
 * legal child of every evaluated position, child_offsets[total positions + 1]
 * indexed by position (as gn_expand_and_evaluate).  GN_E_CAPACITY when the
 * positions exceed position_cap or the children child_cap (the offsets are still
 * filled so the caller can retry with the right sizes). */
GN_API int gn_evaluate_games(gn_ctx *ctx, const gn_game *games, size_t n_games, int mode, int with_children,
                             uint32_t *position_offsets, int32_t *game_status, gn_eval *position_out,
                             size_t position_cap, uint32_t *child_offsets, uint16_t *child_moves,
                             gn_child *child_out, size_t child_cap);

/* The partitioner the library uses to shard work over the devices of a context and
 * that multi-process callers use to shard over ranks: contiguous ranges of n_items
 * items, bounds[k] = first item of shard k, bounds[n_shards] = n_items; shard k
 * starts at the first item whose weight prefix reaches ceil(k * total / n_shards)
 * (weights NULL: every item weighs 1).  gn_evaluate_games shards games weighted
 * by evaluated positions; gn_expand_and_evaluate / gn_evaluate_batch shard parents /
 * positions equally.  Host only. */
GN_API int gn_partition(const uint32_t *weights, size_t n_items, int n_shards, size_t *bounds);

/* Legal-move-tree node count from fen to depth (GPU movegen, breadth-first). */
GN_API int gn_perft(gn_ctx *ctx, const char *fen, int depth, uint64_t *nodes);

/* ---- packed / device-resident API (benchmarks, multi-GPU shards) -------- */
/* Host FEN -> packed board; ok[i] = 0 marks a bad FEN (its board is zeroed).
 * Needs no context and no GPU. */
GN_API int gn_pack_fens(const char *const *fens, size_t n, gn_board *out, uint8_t *ok);
/* Packed board -> FEN text (Chess960-aware X-FEN castling); buf >= 100 bytes. */
GN_API int gn_board_to_fen(const gn_board *board, char *buf, size_t buflen);
/* n boards -> n NUL-terminated FENs at buf + i * stride (stride >= 100); an invalid
 * board gives "".  Host only, multithreaded. */
GN_API int gn_boards_to_fens(const gn_board *boards, size_t n, char *buf, size_t stride);
/* Deterministic random-playout positions (xoshiro256**, seed + index): plays
 * k ~ U{0..max_plies} uniformly random legal plies from the start position
 * (stopping at mate/stalemate), resampling positions in check. Host only. */
GN_API int gn_random_positions(uint64_t seed, size_t first_index, size_t n, int max_plies, gn_board *out);

/* Same generator on the GPU (identical boards for identical seeds): writes n
 * boards to device memory d_out; asynchronous on `stream` (NULL = context stream). */
GN_API int gn_random_positions_device(gn_ctx *ctx, int device_slot, uint64_t seed, size_t first_index, size_t n,
                                      int max_plies, gn_board *d_out, void *stream);

/* Evaluate boards already resident on device `device_slot` (index into the
 * devices given at load).  d_boards / d_out are device pointers; stream is a
 * hipStream_t (NULL = the context's own stream).  Blocking: the score rule reads the
 * number of in-check positions back to size its launches (so the call synchronises
 * `stream` while it runs and cannot be captured into a HIP graph), and the call returns
 * with `stream` idle and d_out written.  The other gn_*_device calls that evaluate
 * (gn_expand_device, gn_expand2_device, gn_time_*) block the same way;
 * gn_random_positions_device / gn_random_games_device are asynchronous. */
GN_API int gn_evaluate_device(gn_ctx *ctx, int device_slot, const gn_board *d_boards, size_t n, int mode,
                       gn_eval *d_out, void *stream);
/* Device-resident expansion: counts children (d_counts[n]), writes d_offsets
 * (n+1 prefix sums), the child boards, moves and evaluations.  Synchronous;
 * returns the total child count in *total. */
GN_API int gn_expand_device(gn_ctx *ctx, int device_slot, const gn_board *d_parents, size_t n, int mode,
                     gn_eval *d_parent_out, uint32_t *d_offsets, gn_board *d_children,
                     uint16_t *d_moves, gn_eval *d_child_out, size_t cap, size_t *total, void *stream);
/* Time `iters` complete expansions of device-resident parents (child count +
 * scan + child generation with deltas + evaluation of parents and children in
 * `mode` + the parents' score rule).  Outputs go to the caller's device buffers when given (d_parent_out[n],
 * d_offsets[n + 1], d_moves[cap], d_child_out[cap]; GN_E_CAPACITY when the
 * children exceed cap), else to library-owned buffers; every iteration writes the
 * same values, so after the call they hold the timed expansion's results.
 * *total = children per expansion;
 * stage_ms (optional, length 8) = average ms of [count+scan, total read-back,
 * write children, classify, small net, big net, finalize, score rule]; ft_rows (optional)
 * = feature-transformer rows one incremental expansion gathers: for the big
 * nets the row stream's own count (bias, carry and king-cache rows included:
 * GN_OPT_CHAIN, GN_OPT_KING_CACHE), else parent refreshes + child deltas /
 * king-move refreshes; 0 when not incremental. */
/* Depth 2 (grandchildren): gn_expand_device, then every child's legal children
 * evaluated incrementally from the child's accumulator (a sibling block refreshes each
 * child from its predecessor through the king cache).  d_goffsets: total + 1 offsets of
 * each child's grandchildren in d_gmoves / d_grand_out (gcap entries); grandchild boards
 * are not returned.  GN_E_CAPACITY: *total / *gtotal hold the counts needed. */
GN_API int gn_expand2_device(gn_ctx *ctx, int device_slot, const gn_board *d_parents, size_t n, int mode,
                             gn_eval *d_parent_out, uint32_t *d_offsets, gn_board *d_children, uint16_t *d_moves,
                             gn_eval *d_child_out, size_t cap, uint32_t *d_goffsets, uint16_t *d_gmoves,
                             gn_eval *d_grand_out, size_t gcap, size_t *total, size_t *gtotal, void *stream);
GN_API int gn_time_expand_device(gn_ctx *ctx, int device_slot, const gn_board *d_parents, size_t n, int mode,
                                 int iters, float *ms_total, size_t *total, float *stage_ms, uint64_t *ft_rows,
                                 gn_eval *d_parent_out, uint32_t *d_offsets, uint16_t *d_moves,
                                 gn_eval *d_child_out, size_t cap);
/* *sum = position-sensitive 64-bit checksum of `bytes` bytes at device pointer d_ptr
 * (sum over 8-byte words w_i of splitmix64(w_i ^ i * 0x9E3779B97F4A7C15), wrapping):
 * compares large device-resident results without a download. */
GN_API int gn_checksum_device(gn_ctx *ctx, int device_slot, const void *d_ptr, size_t bytes, uint64_t *sum);
/* n_games random games of `plies` plies (xoshiro256**, seed + game index) on
 * the GPU: d_out[g * (plies + 1) + k] = position after k plies of game g (a
 * game that ends early repeats its final position).  Asynchronous. */
GN_API int gn_random_games_device(gn_ctx *ctx, int device_slot, uint64_t seed, size_t first_game, size_t n_games,
                                  int plies, gn_board *d_out, void *stream);
/* The UCI moves of the same games gn_random_games_device plays, as the lichess API sends a
 * game (AcquireResponseBody.moves: space-separated, standard castling notation e1g1): game g's
 * NUL-terminated string at buf + g * stride (stride >= 6 * plies + 1); a game that ended
 * (mate, stalemate, rule50) stops there.  Host only, multithreaded. */
GN_API int gn_random_games_uci(uint64_t seed, size_t first_game, size_t n_games, int plies, char *buf, size_t stride);
/* Device memory helpers (so callers need no HIP headers). */
GN_API int gn_device_alloc(gn_ctx *ctx, int device_slot, size_t bytes, void **ptr);
GN_API int gn_device_free(gn_ctx *ctx, int device_slot, void *ptr);
GN_API int gn_memcpy_h2d(gn_ctx *ctx, int device_slot, void *dst, const void *src, size_t bytes);
GN_API int gn_memcpy_d2h(gn_ctx *ctx, int device_slot, void *dst, const void *src, size_t bytes);
GN_API int gn_synchronize(gn_ctx *ctx, int device_slot);
/* Time `iters` back-to-back gn_evaluate_device calls with HIP events recorded
 * on the launch stream; *ms_total = elapsed time.  per_kernel_ms (optional,
 * length 4) receives the average per-call time of the [classify(+reeval),
 * small net, big net, finalize] stages, from events recorded between the
 * launches of that same timed pass (one host sync at the end).  ft_rows
 * (optional) = feature-transformer rows one call's gather reads (the big net's,
 * or the small net's in GN_MODE_SMALL), counted by the kernel. */
GN_API int gn_time_evaluate_device(gn_ctx *ctx, int device_slot, const gn_board *d_boards, size_t n, int mode,
                            gn_eval *d_out, int iters, float *ms_total, float *per_kernel_ms, uint64_t *ft_rows);

#ifdef __cplusplus
}
#endif
#endif
