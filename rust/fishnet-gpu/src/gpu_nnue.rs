//! src/gpu_nnue.rs of the fishnet crate: the safe wrapper over `gpu-nnue-sys`.
//!
//! Drop this file into fishnet's `src/` (`mod gpu_nnue;` in main.rs) and add
//! `gpu-nnue-sys = { path = "..." }` to its Cargo.toml.  The unsafe
//! blocks stay here: fishnet's own `#![forbid(unsafe_code)]` (src/main.rs:1) covers the
//! binary's modules, so this module carries an `#[allow(unsafe_code)]` at its `mod` line
//! in main.rs, or lives in a small library crate beside the -sys crate.
//!
//! Boundary (include/gpu_nnue.h): a `GpuNnue` owns one `gn_ctx`; the library serialises
//! calls on a context, so `&self` methods are safe to share across threads; call them
//! from `tokio::task::spawn_blocking` (the worker runtime is current_thread,
//! /root/reference/src/main.rs:44).
use std::{
    ffi::{CStr, CString},
    path::Path,
    ptr,
};

use gpu_nnue_sys as sys;
use shakmaty::{fen::Fen, uci::UciMove, Role, Square};

pub use sys::gn_child as GpuChild;
pub use sys::gn_eval as GpuEval;

pub struct GpuNnue(*mut sys::gn_ctx);

// SAFETY: the library serialises every call on one context internally (gpu_nnue.h).
unsafe impl Send for GpuNnue {}
unsafe impl Sync for GpuNnue {}

#[derive(Debug, Clone)]
pub struct GpuError {
    pub code: i32,
    pub message: String,
}

impl std::fmt::Display for GpuError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "gpu_nnue error {}: {}", self.code, self.message)
    }
}

impl std::error::Error for GpuError {}

fn last_error(code: i32) -> GpuError {
    // SAFETY: gn_last_error returns a thread-local, NUL-terminated string.
    let message = unsafe { CStr::from_ptr(sys::gn_last_error()) }.to_string_lossy().into_owned();
    GpuError { code, message }
}

fn check(code: i32) -> Result<(), GpuError> {
    if code == sys::GN_OK {
        Ok(())
    } else {
        Err(last_error(code))
    }
}

fn cpath(p: &Path) -> CString {
    CString::new(p.as_os_str().as_encoded_bytes()).expect("path without NUL")
}

/// Every position plus every legal child (gn_evaluate_games with_children = 1).
pub struct GamesResult {
    pub position_offsets: Vec<u32>, // per game, into `positions`
    pub game_status: Vec<i32>,      // GN_OK or GN_E_ILLEGAL_MOVE per game
    pub positions: Vec<GpuEval>,
    pub child_offsets: Vec<u32>, // per position, into `children`
    pub child_moves: Vec<u16>,   // Stockfish move encoding
    pub children: Vec<GpuChild>, // (psqt, positional, final_cp + flags), ABI v4
}

impl GpuNnue {
    /// The two nets as files: nn-1c0000000000.nnue (big) and nn-37f18f62d772.nnue
    /// (small) (/root/reference/build.rs:8-9).
    pub fn load_net(big: &Path, small: &Path, devices: &[i32]) -> Result<GpuNnue, GpuError> {
        let (b, s) = (cpath(big), cpath(small));
        let mut ctx = ptr::null_mut();
        // SAFETY: valid C strings and an out pointer; devices may be empty (device 0).
        check(unsafe {
            sys::gn_load_net(b.as_ptr(), s.as_ptr(), devices.as_ptr(), devices.len() as i32, &mut ctx)
        })?;
        Ok(GpuNnue(ctx))
    }

    /// Both nets straight out of fishnet's embedded assets.ar.zst (the archive
    /// Assets::prepare reads, /root/reference/src/assets.rs:186-226), written once to a
    /// file; the first big and the first small .nnue member are taken.
    pub fn load_net_archive(archive: &Path, devices: &[i32]) -> Result<GpuNnue, GpuError> {
        let a = cpath(archive);
        let mut ctx = ptr::null_mut();
        // SAFETY: as above; NULL member names select by kind.
        check(unsafe {
            sys::gn_load_net_archive(a.as_ptr(), ptr::null(), ptr::null(), devices.as_ptr(), devices.len() as i32,
                                     &mut ctx)
        })?;
        Ok(GpuNnue(ctx))
    }

    /// evaluate_batch(&[Fen]) -> (psqt, positional, final_v, final_cp) per position,
    /// side-to-move POV, plus the score fishnet posts (score / GN_FLAG_MATE / best_move:
    /// checkmate, stalemate and checks included, include/gpu_nnue.h at gn_eval).
    pub fn evaluate_batch(&self, fens: &[Fen]) -> Result<Vec<GpuEval>, GpuError> {
        let owned: Vec<CString> = fens.iter().map(|f| CString::new(f.to_string()).unwrap()).collect();
        let ptrs: Vec<*const std::os::raw::c_char> = owned.iter().map(|c| c.as_ptr()).collect();
        let mut out = vec![GpuEval::default(); fens.len()];
        // SAFETY: ptrs / out have fens.len() elements and outlive the call.
        check(unsafe { sys::gn_evaluate_batch(self.0, ptrs.as_ptr(), ptrs.len(), out.as_mut_ptr()) })?;
        Ok(out)
    }

    /// Whole acquired batches: replay root FEN + UCI moves (skipPositions honoured) and
    /// evaluate every position and every legal child; buffers grow on GN_E_CAPACITY.
    pub fn evaluate_games(&self, games: &[(CString, CString, Vec<u32>)], mode: i32) -> Result<GamesResult, GpuError> {
        let gs: Vec<sys::gn_game> = games
            .iter()
            .map(|(root, moves, skip)| sys::gn_game {
                root_fen: root.as_ptr(),
                uci_moves: moves.as_ptr(),
                skip_positions: skip.as_ptr(),
                n_skip: skip.len(),
            })
            .collect();
        let (mut pcap, mut ccap) = (games.len() * 128, games.len() * 128 * 40);
        loop {
            let mut r = GamesResult {
                position_offsets: vec![0; games.len() + 1],
                game_status: vec![0; games.len()],
                positions: vec![GpuEval::default(); pcap],
                child_offsets: vec![0; pcap + 1],
                child_moves: vec![0; ccap],
                children: vec![GpuChild::default(); ccap],
            };
            // SAFETY: every buffer has the length the call is told.
            let rc = unsafe {
                sys::gn_evaluate_games(self.0, gs.as_ptr(), gs.len(), mode, 1, r.position_offsets.as_mut_ptr(),
                                       r.game_status.as_mut_ptr(), r.positions.as_mut_ptr(), pcap,
                                       r.child_offsets.as_mut_ptr(), r.child_moves.as_mut_ptr(),
                                       r.children.as_mut_ptr(), ccap)
            };
            if rc == sys::GN_E_CAPACITY {
                // the offsets hold the sizes needed
                pcap = pcap.max(*r.position_offsets.last().unwrap() as usize);
                let np = (*r.position_offsets.last().unwrap() as usize).min(r.child_offsets.len() - 1);
                ccap = ccap.max(r.child_offsets[np] as usize).max(ccap * 2);
                continue;
            }
            check(rc)?;
            let np = *r.position_offsets.last().unwrap() as usize;
            let nc = r.child_offsets[np] as usize;
            r.positions.truncate(np);
            r.child_offsets.truncate(np + 1);
            r.child_moves.truncate(nc);
            r.children.truncate(nc);
            return Ok(r);
        }
    }
}

/// A move in Stockfish's 16-bit encoding (gn_eval.best_move, child_moves) as the Chess960 UCI
/// fishnet runs its engines with (castling = king takes rook, stockfish.rs:200).
pub fn move_to_uci(m: u16) -> UciMove {
    const PROMO: [Role; 4] = [Role::Knight, Role::Bishop, Role::Rook, Role::Queen];
    UciMove::Normal {
        from: Square::new(u32::from((m >> 6) & 63)),
        to: Square::new(u32::from(m & 63)),
        promotion: (m >> 14 == 1).then(|| PROMO[usize::from((m >> 12) & 3)]),
    }
}

impl Drop for GpuNnue {
    fn drop(&mut self) {
        // SAFETY: the context was created by gn_load_net* and is freed once.
        unsafe { sys::gn_free(self.0) }
    }
}
