//! gpu-nnue-sys — raw FFI of libgpu_nnue.so, 1:1 with `include/gpu_nnue.h` (ABI v4).
//!
//! fishnet's `src/main.rs:1` forbids unsafe code in the binary crate, so the FFI lives in
//! this separate crate; the safe wrapper is `fishnet-gpu/src/gpu_nnue.rs`.  Every item here
//! mirrors a declaration of the header; `tests/test_host.py::test_rust_sys_crate_matches_header`
//! checks names, argument counts, struct fields and constants against it (cargo is not
//! in the build image, so that test is what keeps this file honest).
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

pub const GN_ABI_VERSION: c_int = 4;

// return codes
pub const GN_OK: c_int = 0;
pub const GN_E_INVALID: c_int = -1;
pub const GN_E_IO: c_int = -2;
pub const GN_E_FORMAT: c_int = -3;
pub const GN_E_HIP: c_int = -4;
pub const GN_E_NOMEM: c_int = -5;
pub const GN_E_CAPACITY: c_int = -6;
pub const GN_E_NODEVICE: c_int = -7;
pub const GN_E_NONET: c_int = -8;
pub const GN_E_ILLEGAL_MOVE: c_int = -9;

// evaluation modes
pub const GN_MODE_FULL: c_int = 0;
pub const GN_MODE_BIG: c_int = 1;
pub const GN_MODE_SMALL: c_int = 2;

// options (gn_set_option / gn_get_option); results never depend on them
pub const GN_OPT_INCREMENTAL_CHILDREN: c_int = 1;
pub const GN_OPT_XCD_SWIZZLE: c_int = 2;
pub const GN_OPT_KING_SORT: c_int = 3;
pub const GN_OPT_CHAIN: c_int = 4;
pub const GN_OPT_KING_CACHE: c_int = 5;
pub const GN_OPT_CHUNK_PARENTS: c_int = 6;
pub const GN_OPT_COALESCE: c_int = 7;
pub const GN_OPT_STREAM_SLICES: c_int = 8;
pub const GN_OPT_FAST_BATCH: c_int = 9;
pub const GN_OPT_EXPAND_PIPELINE: c_int = 10;
// read-only statistics (gn_get_option)
pub const GN_STAT_PLAN_NS: c_int = 101;
pub const GN_STAT_STREAM_NS: c_int = 102;
pub const GN_STAT_SCRATCH_PADS: c_int = 103;
pub const GN_STAT_FINISH_NS: c_int = 104;
pub const GN_STAT_HOST_PARSE_NS: c_int = 110;
pub const GN_STAT_HOST_UPLOAD_NS: c_int = 111;
pub const GN_STAT_HOST_REPLAY_NS: c_int = 112;
pub const GN_STAT_HOST_COMPUTE_NS: c_int = 113;
pub const GN_STAT_HOST_DOWNLOAD_NS: c_int = 114;
pub const GN_STAT_HOST_TAIL_NS: c_int = 115;
pub const GN_STAT_HOST_TOTAL_NS: c_int = 116;
pub const GN_STAT_BATCH_LAUNCHES: c_int = 117;
pub const GN_STAT_BATCH_CALLS: c_int = 118;
pub const GN_STAT_FAST_BATCHES: c_int = 119;
pub const GN_STAT_FAST_FALLBACKS: c_int = 120;

// per-position flags
pub const GN_FLAG_IN_CHECK: u16 = 1;
pub const GN_FLAG_SMALLNET: u16 = 2;
pub const GN_FLAG_BAD_FEN: u16 = 4;
pub const GN_FLAG_REEVAL: u16 = 8;
pub const GN_FLAG_SKIPPED: u16 = 16;
pub const GN_FLAG_MATE: u16 = 32;
pub const GN_FLAG_NO_SCORE: u16 = 64;
pub const GN_FLAG_SEARCHED: u16 = 128;
pub const GN_FLAG_NO_MOVES: u16 = 256;

/// One result: NetworkOutput (psqt, positional) of the net that produced final_v,
/// Eval::evaluate (internal units), UCIEngine::to_cp, and the score fishnet posts for the
/// position (`score cp` / `score mate` with GN_FLAG_MATE; the in-check rule's reply in
/// best_move with GN_FLAG_SEARCHED; see the header at gn_eval).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct gn_eval {
    pub psqt: i32,
    pub positional: i32,
    pub final_v: i32,
    pub final_cp: i32,
    pub score: i32,
    pub flags: u16,
    pub best_move: u16,
}

/// One legal child from the host-buffer expansion calls (ABI v4, 12 bytes): psqt, positional and
/// cp_flags = final_cp (signed 24 bits) | the low 8 flag bits << 24 (see the header at gn_child).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct gn_child {
    pub psqt: i32,
    pub positional: i32,
    pub cp_flags: i32,
}

impl gn_child {
    /// GN_CHILD_FINAL_CP
    pub fn final_cp(&self) -> i32 {
        ((self.cp_flags as u32) << 8) as i32 >> 8
    }
    /// GN_CHILD_FLAGS
    pub fn flags(&self) -> u16 {
        ((self.cp_flags as u32) >> 24) as u16
    }
}

/// Packed position (32 bytes), the device input format.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct gn_board {
    pub occ: u64,
    pub pc: [u8; 16],
    pub stm_ep: u8,
    pub reserved: u8,
    pub castle: u16,
    pub rule50: u16,
    pub fullmove: u16,
}

/// Eval::evaluate constants and the to_cp win-rate model (defaults: Stockfish 17.1).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq)]
pub struct gn_eval_params {
    pub small_net_threshold: i32,
    pub psqt_weight: i32,
    pub positional_weight: i32,
    pub reeval_threshold: i32,
    pub complexity_div_small: i32,
    pub complexity_div_big: i32,
    pub material_pawn_small: i32,
    pub material_pawn_big: i32,
    pub material_base: i32,
    pub rule50_div: i32,
    pub value_clamp: i32,
    pub piece_value: [i32; 5],
    pub wdl_a: [f64; 4],
    pub wdl_material_min: i32,
    pub wdl_material_max: i32,
    pub wdl_material_anchor: i32,
    pub wdl_piece_weight: [i32; 5],
}

/// One acquired lichess batch (AcquireResponseBody, src/api.rs:306-321).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct gn_game {
    pub root_fen: *const c_char,
    pub uci_moves: *const c_char,
    pub skip_positions: *const u32,
    pub n_skip: usize,
}

#[repr(C)]
pub struct gn_ctx {
    _private: [u8; 0],
}

#[link(name = "gpu_nnue")]
extern "C" {
    pub fn gn_load_net(big_path: *const c_char, small_path: *const c_char, devices: *const c_int, n_devices: c_int,
                       out: *mut *mut gn_ctx) -> c_int;
    pub fn gn_load_net_memory(big: *const u8, big_len: usize, small: *const u8, small_len: usize,
                              devices: *const c_int, n_devices: c_int, out: *mut *mut gn_ctx) -> c_int;
    pub fn gn_load_net_archive(archive_path: *const c_char, big_member: *const c_char, small_member: *const c_char,
                               devices: *const c_int, n_devices: c_int, out: *mut *mut gn_ctx) -> c_int;
    pub fn gn_archive_read(archive_path: *const c_char, member: *const c_char, buf: *mut u8, cap: usize,
                           size: *mut usize) -> c_int;
    pub fn gn_free(ctx: *mut gn_ctx);
    pub fn gn_last_error() -> *const c_char;
    pub fn gn_abi_version() -> c_int;
    pub fn gn_get_eval_params(ctx: *const gn_ctx, out: *mut gn_eval_params) -> c_int;
    pub fn gn_set_eval_params(ctx: *mut gn_ctx, params: *const gn_eval_params) -> c_int;
    pub fn gn_set_option(ctx: *mut gn_ctx, option: c_int, value: i64) -> c_int;
    pub fn gn_get_option(ctx: *const gn_ctx, option: c_int, value: *mut i64) -> c_int;
    pub fn gn_net_sha256(data: *const u8, len: usize, hex65: *mut c_char) -> c_int;
    pub fn gn_net_info(ctx: *const gn_ctx, big_l1: *mut c_int, big_hash: *mut u32, small_l1: *mut c_int,
                       small_hash: *mut u32) -> c_int;
    pub fn gn_evaluate_batch(ctx: *mut gn_ctx, fens: *const *const c_char, n: usize, out: *mut gn_eval) -> c_int;
    pub fn gn_evaluate_batch_mode(ctx: *mut gn_ctx, fens: *const *const c_char, n: usize, mode: c_int,
                                  out: *mut gn_eval) -> c_int;
    pub fn gn_expand_and_evaluate(ctx: *mut gn_ctx, parent_fens: *const *const c_char, n: usize, mode: c_int,
                                  parent_out: *mut gn_eval, child_offsets: *mut u32, child_moves: *mut u16,
                                  child_out: *mut gn_child, cap: usize) -> c_int;
    pub fn gn_replay_game(game: *const gn_game, positions: *mut gn_board, skipped: *mut u8, moves: *mut u16,
                          cap: usize, n_positions: *mut usize) -> c_int;
    pub fn gn_evaluate_games(ctx: *mut gn_ctx, games: *const gn_game, n_games: usize, mode: c_int,
                             with_children: c_int, position_offsets: *mut u32, game_status: *mut i32,
                             position_out: *mut gn_eval, position_cap: usize, child_offsets: *mut u32,
                             child_moves: *mut u16, child_out: *mut gn_child, child_cap: usize) -> c_int;
    pub fn gn_partition(weights: *const u32, n_items: usize, n_shards: c_int, bounds: *mut usize) -> c_int;
    pub fn gn_perft(ctx: *mut gn_ctx, fen: *const c_char, depth: c_int, nodes: *mut u64) -> c_int;
    pub fn gn_pack_fens(fens: *const *const c_char, n: usize, out: *mut gn_board, ok: *mut u8) -> c_int;
    pub fn gn_board_to_fen(board: *const gn_board, buf: *mut c_char, buflen: usize) -> c_int;
    pub fn gn_boards_to_fens(boards: *const gn_board, n: usize, buf: *mut c_char, stride: usize) -> c_int;
    pub fn gn_random_positions(seed: u64, first_index: usize, n: usize, max_plies: c_int, out: *mut gn_board)
                               -> c_int;
    // device-resident entry points (pointers are device memory of device_slot; stream: a
    // hipStream_t or NULL for the library's own)
    pub fn gn_random_positions_device(ctx: *mut gn_ctx, device_slot: c_int, seed: u64, first_index: usize, n: usize,
                                      max_plies: c_int, d_out: *mut gn_board, stream: *mut c_void) -> c_int;
    pub fn gn_evaluate_device(ctx: *mut gn_ctx, device_slot: c_int, d_boards: *const gn_board, n: usize, mode: c_int,
                              d_out: *mut gn_eval, stream: *mut c_void) -> c_int;
    pub fn gn_expand_device(ctx: *mut gn_ctx, device_slot: c_int, d_parents: *const gn_board, n: usize, mode: c_int,
                            d_parent_out: *mut gn_eval, d_offsets: *mut u32, d_children: *mut gn_board,
                            d_moves: *mut u16, d_child_out: *mut gn_eval, cap: usize, total: *mut usize,
                            stream: *mut c_void) -> c_int;
    pub fn gn_expand2_device(ctx: *mut gn_ctx, device_slot: c_int, d_parents: *const gn_board, n: usize, mode: c_int,
                             d_parent_out: *mut gn_eval, d_offsets: *mut u32, d_children: *mut gn_board,
                             d_moves: *mut u16, d_child_out: *mut gn_eval, cap: usize, d_goffsets: *mut u32,
                             d_gmoves: *mut u16, d_grand_out: *mut gn_eval, gcap: usize, total: *mut usize,
                             gtotal: *mut usize, stream: *mut c_void) -> c_int;
    pub fn gn_time_expand_device(ctx: *mut gn_ctx, device_slot: c_int, d_parents: *const gn_board, n: usize,
                                 mode: c_int, iters: c_int, ms_total: *mut f32, total: *mut usize,
                                 stage_ms: *mut f32, ft_rows: *mut u64, d_parent_out: *mut gn_eval,
                                 d_offsets: *mut u32, d_moves: *mut u16, d_child_out: *mut gn_eval, cap: usize)
                                 -> c_int;
    pub fn gn_checksum_device(ctx: *mut gn_ctx, device_slot: c_int, d_ptr: *const c_void, bytes: usize,
                              sum: *mut u64) -> c_int;
    pub fn gn_random_games_device(ctx: *mut gn_ctx, device_slot: c_int, seed: u64, first_game: usize,
                                  n_games: usize, plies: c_int, d_out: *mut gn_board, stream: *mut c_void) -> c_int;
    pub fn gn_random_games_uci(seed: u64, first_game: usize, n_games: usize, plies: c_int, buf: *mut c_char,
                               stride: usize) -> c_int;
    pub fn gn_device_alloc(ctx: *mut gn_ctx, device_slot: c_int, bytes: usize, ptr: *mut *mut c_void) -> c_int;
    pub fn gn_device_free(ctx: *mut gn_ctx, device_slot: c_int, ptr: *mut c_void) -> c_int;
    pub fn gn_memcpy_h2d(ctx: *mut gn_ctx, device_slot: c_int, dst: *mut c_void, src: *const c_void, bytes: usize)
                         -> c_int;
    pub fn gn_memcpy_d2h(ctx: *mut gn_ctx, device_slot: c_int, dst: *mut c_void, src: *const c_void, bytes: usize)
                         -> c_int;
    pub fn gn_synchronize(ctx: *mut gn_ctx, device_slot: c_int) -> c_int;
    pub fn gn_time_evaluate_device(ctx: *mut gn_ctx, device_slot: c_int, d_boards: *const gn_board, n: usize,
                                   mode: c_int, d_out: *mut gn_eval, iters: c_int, ms_total: *mut f32,
                                   per_kernel_ms: *mut f32, ft_rows: *mut u64) -> c_int;
}

#[cfg(test)]
mod tests {
    use super::*;
    #[test]
    fn layouts() {
        assert_eq!(std::mem::size_of::<gn_eval>(), 24);
        assert_eq!(std::mem::size_of::<gn_child>(), 12);
        let c = gn_child { psqt: 0, positional: 0, cp_flags: (0x00FF_FFFEu32 | 65u32 << 24) as i32 };
        assert_eq!((c.final_cp(), c.flags()), (-2, 65));
        assert_eq!(std::mem::size_of::<gn_board>(), 32);
        assert_eq!(std::mem::size_of::<gn_eval_params>(), 128);
    }
}
