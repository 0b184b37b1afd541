//! The GPU backend beside `StockfishStub` (/root/reference/src/stockfish.rs:32-47): the
//! same `go_multiple(Chunk) -> Result<Vec<PositionResponse>, ChunkFailed>` signature, so
//! the worker's `tokio::select!` (src/main.rs:267-303) can call either.  Goes into
//! fishnet's src/stockfish.rs (or a sibling module) beside StockfishStub.
use std::{num::NonZeroU8, sync::Arc, time::Duration};

use shakmaty::{fen::Fen, uci::UciMove, CastlingMode, Chess, EnPassantMode, Position as _};

use crate::{
    api::Score,
    gpu_nnue::GpuNnue,
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

impl GpuEvalStub {
    pub fn new(nnue: Arc<GpuNnue>) -> GpuEvalStub {
        GpuEvalStub { nnue }
    }

    pub async fn go_multiple(&mut self, chunk: Chunk) -> Result<Vec<PositionResponse>, ChunkFailed> {
        let batch_id = chunk.work.id();
        let fens: Vec<Option<Fen>> = chunk.positions.iter().map(replay_to_fen).collect();
        if fens.iter().any(Option::is_none) {
            return Err(ChunkFailed { batch_id }); // an illegal move, as queue.rs:576 fails the batch
        }
        let fens: Vec<Fen> = fens.into_iter().flatten().collect();
        let nnue = self.nnue.clone();
        let evals = tokio::task::spawn_blocking(move || nnue.evaluate_batch(&fens))
            .await
            .map_err(|_| ChunkFailed { batch_id })?
            .map_err(|_| ChunkFailed { batch_id })?; // GN_E_* -> ChunkFailed (the existing drop path)
        Ok(chunk
            .positions
            .into_iter()
            .zip(evals)
            .map(|(pos, e)| {
                let mut scores = Matrix::new();
                if pos.skip {
                    // skipPositions: no score, as the UCI path leaves them
                } else if e.flags & (sys::GN_FLAG_IN_CHECK | sys::GN_FLAG_BAD_FEN) == 0 {
                    // static eval, no search: the centipawns Stockfish prints (UCIEngine::to_cp),
                    // i.e. what stockfish.rs:419-427 parses from `score cp`
                    scores.set(NonZeroU8::MIN, 0, Score::Cp(i64::from(e.final_cp)));
                }
                PositionResponse {
                    work: pos.work,
                    position_index: pos.position_index,
                    url: pos.url,
                    scores,
                    pvs: Matrix::new(),
                    best_move: None::<UciMove>,
                    depth: 0,
                    nodes: 1,
                    time: Duration::ZERO,
                    nps: None,
                }
            })
            .collect())
    }
}
