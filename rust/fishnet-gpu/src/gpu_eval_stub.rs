//! The GPU backend beside `StockfishStub` (/root/reference/src/stockfish.rs:32-47): the
//! same `go_multiple(Chunk) -> Result<Vec<PositionResponse>, ChunkFailed>` signature, so
//! the worker's `tokio::select!` (src/main.rs:267-303) can call either.  Goes into
//! fishnet's src/stockfish.rs (or a sibling module) beside StockfishStub.
//!
//! Every response carries a score, as Stockfish's `go` always prints one
//! (stockfish.rs:366-368 rejects a response without one, and the queue's
//! `PositionResponse::to_best` does `expect("got score")`, src/ipc.rs:56): the library
//! scores every position it is given (include/gpu_nnue.h at gn_eval): checkmate
//! `mate 0`, stalemate `cp 0`, a position in check by its in-check rule over the legal
//! replies (depth 1, the reply as best move and pv), else the static evaluation's `cp`.
//! This stub only maps those fields; a record without a score (a position the library
//! refuses) fails the chunk like an engine error, never the queue.
use std::{num::NonZeroU8, sync::Arc, time::Duration};

use shakmaty::{fen::Fen, uci::UciMove, CastlingMode, Chess, EnPassantMode, Position as _};

use crate::{
    api::Score,
    gpu_nnue::{move_to_uci, GpuEval, GpuNnue},
    ipc::{Chunk, ChunkFailed, Matrix, Position, PositionResponse},
};
use gpu_nnue_sys as sys;

pub struct GpuEvalStub {
    nnue: Arc<GpuNnue>,
}

/// root FEN + UCI moves -> the FEN to evaluate, replayed like IncomingBatch::from_acquired
/// (/root/reference/src/queue.rs:572-581: shakmaty UciMove::to_move + play_unchecked).
fn replay_to_fen(pos: &Position) -> Option<Fen> {
    let mut board: Chess = pos.root_fen.clone().into_position(CastlingMode::Chess960).ok()?;
    for uci in &pos.moves {
        let m = uci.to_move(&board).ok()?;
        board.play_unchecked(&m);
    }
    Some(Fen::from_position(board, EnPassantMode::Legal))
}

/// The FENs of a whole chunk with one replay: a chunk's positions share their root and their
/// move lists are prefixes of the longest one (IncomingBatch::from_acquired makes position i
/// = root + moves[..i], queue.rs:605-637), so replaying the longest list once yields every
/// position's FEN (O(L) moves instead of the O(L^2) of a replay per position); a position
/// outside that pattern is replayed on its own.  None: a move that does not replay; an empty
/// chunk gives an empty list.
fn replay_chunk(positions: &[Position]) -> Option<Vec<Fen>> {
    if positions.is_empty() {
        return Some(Vec::new()); // an empty chunk is an empty result, not a failed replay
    }
    let longest = positions.iter().max_by_key(|p| p.moves.len())?;
    let mut board: Chess = longest.root_fen.clone().into_position(CastlingMode::Chess960).ok()?;
    let mut line = vec![Fen::from_position(board.clone(), EnPassantMode::Legal)];
    for uci in &longest.moves {
        let m = uci.to_move(&board).ok()?;
        board.play_unchecked(&m);
        line.push(Fen::from_position(board.clone(), EnPassantMode::Legal));
    }
    positions
        .iter()
        .map(|p| {
            if p.root_fen == longest.root_fen && longest.moves.starts_with(&p.moves) {
                Some(line[p.moves.len()].clone())
            } else {
                replay_to_fen(p)
            }
        })
        .collect()
}

/// The score Stockfish would print for the record (`score cp` / `score mate`), or None for a
/// record the library could not score.
pub fn score_of(e: &GpuEval) -> Option<Score> {
    if e.flags & sys::GN_FLAG_NO_SCORE != 0 {
        None
    } else if e.flags & sys::GN_FLAG_MATE != 0 {
        Some(Score::Mate(i64::from(e.score)))
    } else {
        Some(Score::Cp(i64::from(e.score)))
    }
}

impl GpuEvalStub {
    pub fn new(nnue: Arc<GpuNnue>) -> GpuEvalStub {
        GpuEvalStub { nnue }
    }

    pub async fn go_multiple(&mut self, chunk: Chunk) -> Result<Vec<PositionResponse>, ChunkFailed> {
        let batch_id = chunk.work.id();
        // an illegal move fails the chunk, as queue.rs:576 fails the batch
        let fens = replay_chunk(&chunk.positions).ok_or(ChunkFailed { batch_id })?;
        let nnue = self.nnue.clone();
        // N workers call at once through the shared context: the library merges their
        // concurrent calls into one launch (GN_OPT_COALESCE, bench.py secondary.dropin)
        let evals = tokio::task::spawn_blocking(move || nnue.evaluate_batch(&fens))
            .await
            .map_err(|_| ChunkFailed { batch_id })?
            .map_err(|_| ChunkFailed { batch_id })?; // GN_E_* -> ChunkFailed (the existing drop path)
        chunk
            .positions
            .into_iter()
            .zip(evals)
            .map(|(pos, e)| {
                // (positions with skip = true are the previous-position dummies the queue adds for
                // hash warm-up, position_index None: scored like any other, their responses are
                // dropped by QueueState::handle_position_responses, queue.rs:201-206)
                let score = score_of(&e).ok_or(ChunkFailed { batch_id })?;
                let searched = e.flags & sys::GN_FLAG_SEARCHED != 0;
                let depth: u8 = if searched { 1 } else { 0 };
                let mut scores = Matrix::new();
                scores.set(NonZeroU8::MIN, depth, score);
                let mut pvs = Matrix::new();
                let best_move: Option<UciMove> = searched.then(|| move_to_uci(e.best_move));
                if let Some(m) = &best_move {
                    pvs.set(NonZeroU8::MIN, depth, vec![m.clone()]);
                }
                Ok(PositionResponse {
                    work: pos.work,
                    position_index: pos.position_index,
                    url: pos.url,
                    scores,
                    pvs,
                    best_move,
                    depth,
                    nodes: 1,
                    time: Duration::ZERO,
                    nps: None,
                })
            })
            .collect()
    }
}
