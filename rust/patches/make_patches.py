#!/usr/bin/env python3
"""Writes rust/patches/*.patch: the changes a fishnet maintainer applies to the reference tree
(ounben/fishnet, /root/reference) to build it with the MI355X GPU evaluation backend.

    python rust/patches/make_patches.py [--check] [--reference /root/reference]

Each patch is a list of exact textual edits applied to a scratch copy of the reference's files,
then `diff -u`: the edits fail loudly if the reference moved.  --check compares the output with
the committed patches instead of writing them (tests/test_host.py runs it and `patch --dry-run`).
Apply with `patch -p1 < rust/patches/<file>` in the fishnet checkout, after copying this repo's
`rust/` to `<fishnet>/gpu/`.

0001-compile-fixes.patch   the reference as mounted does not compile: src/stats.rs imports
                           rusqlite (not in Cargo.toml / Cargo.lock) and deleted
                           StatsRecorder::min_user_backlog, which src/queue.rs:353 calls.  The
                           SQLite writer (a fork addition) goes; min_user_backlog is restored as
                           upstream fishnet has it (recalled: 60-position batches at 2.25 M
                           nodes, top clients ~35 s).
0002-gpu-eval-backend.patch the backend: feature `gpu` (Cargo.toml, gpu-nnue-sys path dependency);
                           `--gpu-devices 0,1,...` (src/configure.rs); nets loaded once from the
                           extracted assets and a GpuEvalStub raced against the chunk deadline
                           for standard-chess analysis chunks in the worker (src/main.rs:263-390);
                           whole batches as one chunk when the GPU takes them
                           (src/queue.rs:548-700, the flavor decision at :562-568 unchanged).
"""
import argparse
import difflib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

STATS = [
    ("src/stats.rs", "    time::{Duration, SystemTime, UNIX_EPOCH},\n", "    time::Duration,\n"),
    ("src/stats.rs", "use rusqlite::{params, Connection, Result}; // SQLite-Bibliothek\n", ""),
    ("src/stats.rs", "    cores: NonZeroUsize,\n    db_conn: Option<Connection>, // SQLite-Verbindung\n}\n",
     "    cores: NonZeroUsize,\n}\n"),
    ("src/stats.rs", "                nnue_nps,\n                cores,\n                db_conn: None,\n            };",
     "                nnue_nps,\n                cores,\n            };"),
    ("src/stats.rs", """        // SQLite-Datenbank initialisieren
        let db_conn = match initialize_database("stats.db") {
            Ok(conn) => Some(conn),
            Err(err) => {
                eprintln!("E: Failed to initialize SQLite database: {err}");
                None
            }
        };

""", ""),
    ("src/stats.rs", "            nnue_nps,\n            cores,\n            db_conn,\n        }\n    }\n",
     "            nnue_nps,\n            cores,\n        }\n    }\n"),
    ("src/stats.rs", """        // Speichern in .stats-file
        if let Some((ref path, ref mut stats_file)) = &self.store {""",
     """        if let Some((ref path, ref mut stats_file)) = &self.store {"""),
    ("src/stats.rs", """
        // Speichern in SQLite-Datenbank
        if let Some(conn) = &self.db_conn {
            if let Err(err) = self.save_to_database(conn, nnue_nps) {
                eprintln!("E: Failed to save stats to SQLite database: {err}");
            }
        }
""", ""),
    ("src/stats.rs", None, ("    // Neue Methode: Stats in SQLite speichern\n", "#[derive(Clone)]\npub struct NpsRecorder {"),
     """    pub fn min_user_backlog(&self) -> Duration {
        // The average batch has 60 positions, analysed with 2_250_000 nodes
        // each. Top end clients take no longer than 35 seconds.
        let best_batch_seconds = 35;

        // Estimate how long this client would take for the next batch,
        // capped at timeout.
        let estimated_batch_seconds = min(
            6 * 60,
            60 * 2_250_000 / self.cores.get() as u64 / u64::from(self.nnue_nps.nps.max(1)),
        );

        // Its worth joining if queue wait time + estimated time < top client
        // time on empty queue.
        Duration::from_secs(estimated_batch_seconds.saturating_sub(best_batch_seconds))
    }
}

"""),
]

GPU = [
    ("Cargo.toml", "[dependencies]\narrayvec = \"0.7\"\n", """[features]
# The MI355X GPU evaluation backend: libgpu_nnue.so through gpu/gpu-nnue-sys (gpu/INTEGRATION.md).
gpu = ["dep:gpu-nnue-sys"]

[dependencies]
gpu-nnue-sys = { path = "gpu/gpu-nnue-sys", optional = true }
arrayvec = "0.7"
"""),
    ("src/main.rs", "#![forbid(unsafe_code)]\n",
     "// forbid cannot be relaxed per module: the FFI wrapper (gpu_nnue) needs an allow.\n#![deny(unsafe_code)]\n"),
    ("src/main.rs", "mod util;\n", """mod util;

// The GPU evaluation backend (feature `gpu`; this repo's rust/ copied to gpu/).
#[cfg(feature = "gpu")]
#[path = "../gpu/fishnet-gpu/src/gpu_eval_stub.rs"]
mod gpu_eval_stub;
#[cfg(feature = "gpu")]
#[allow(unsafe_code)]
#[path = "../gpu/fishnet-gpu/src/gpu_nnue.rs"]
mod gpu_nnue;

/// Which chunks the GPU backend takes (standard-chess analysis, EngineFlavor::Official) and
/// running one, raced against its deadline like an engine; compiled to a no-op without `gpu`.
mod gpu_backend {
    use tokio::sync::mpsc;

    use crate::ipc::{Chunk, ChunkFailed, PositionResponse, Pull};

    #[cfg(feature = "gpu")]
    pub type Handle = Option<std::sync::Arc<crate::gpu_nnue::GpuNnue>>;
    #[cfg(not(feature = "gpu"))]
    pub type Handle = ();

    #[cfg(feature = "gpu")]
    pub fn pick(gpu: &Handle, chunk: &Chunk) -> Handle {
        gpu.as_ref()
            .filter(|_| chunk.flavor == crate::assets::EngineFlavor::Official)
            .cloned()
    }
    #[cfg(not(feature = "gpu"))]
    pub fn pick(_: &Handle, _: &Chunk) -> Option<()> {
        None
    }

    /// None when the worker is shutting down.
    #[cfg(feature = "gpu")]
    pub async fn go(
        nnue: std::sync::Arc<crate::gpu_nnue::GpuNnue>,
        chunk: Chunk,
        tx: &mpsc::Sender<Pull>,
    ) -> Option<Result<Vec<PositionResponse>, ChunkFailed>> {
        let batch_id = chunk.work.id();
        let deadline = chunk.deadline;
        let mut stub = crate::gpu_eval_stub::GpuEvalStub::new(nnue);
        tokio::select! {
            _ = tx.closed() => None,
            _ = tokio::time::sleep_until(deadline) => Some(Err(ChunkFailed { batch_id })),
            res = stub.go_multiple(chunk) => Some(res),
        }
    }
    #[cfg(not(feature = "gpu"))]
    pub async fn go(
        _: (),
        _: Chunk,
        _: &mpsc::Sender<Pull>,
    ) -> Option<Result<Vec<PositionResponse>, ChunkFailed>> {
        None
    }
}
"""),
    ("src/main.rs", """    let cores = opt.cores.unwrap_or(Cores::Auto).number();
    logger.info(&format!("Cores: {cores}"));
""", """    let cores = opt.cores.unwrap_or(Cores::Auto).number();
    logger.info(&format!("Cores: {cores}"));

    // The GPU evaluation backend: both nets from the extracted assets (build.rs:8-9), loaded
    // once on the listed devices and shared by every worker.
    #[cfg(feature = "gpu")]
    let gpu: gpu_backend::Handle = opt.gpu_devices.as_ref().map(|devices| {
        let dir = assets
            .stockfish
            .get(EngineFlavor::Official)
            .parent()
            .expect("assets dir")
            .to_owned();
        let nnue = gpu_nnue::GpuNnue::load_net(
            &dir.join("nn-1c0000000000.nnue"),
            &dir.join("nn-37f18f62d772.nnue"),
            &devices.0,
        )
        .expect("nets loaded on the GPU");
        logger.info(&format!("GPU evaluation backend on devices {:?}", devices.0));
        Arc::new(nnue)
    });
    #[cfg(not(feature = "gpu"))]
    let gpu: gpu_backend::Handle = ();
    #[cfg(feature = "gpu")]
    let gpu_chunks = gpu.is_some();
    #[cfg(not(feature = "gpu"))]
    let gpu_chunks = false;
"""),
    ("src/main.rs", """        cores,
        api,
        opt.max_backoff.unwrap_or_default(),
        logger.clone(),
    );""", """        cores,
        api,
        opt.max_backoff.unwrap_or_default(),
        gpu_chunks,
        logger.clone(),
    );"""),
    ("src/main.rs", """            let tx = tx.clone();
            let logger = logger.clone();
            join_set.spawn(worker(i, assets, tx, logger));""", """            let tx = tx.clone();
            let logger = logger.clone();
            join_set.spawn(worker(i, assets, gpu.clone(), tx, logger));"""),
    ("src/main.rs", "async fn worker(i: usize, assets: Arc<Assets>, tx: mpsc::Sender<Pull>, logger: Logger) {",
     """async fn worker(
    i: usize,
    assets: Arc<Assets>,
    gpu: gpu_backend::Handle,
    tx: mpsc::Sender<Pull>,
    logger: Logger,
) {"""),
    ("src/main.rs", """    loop {
        let responses = if let Some(chunk) = chunk.take() {
            // Ensure engine process is ready.""", """    loop {
        let gpu_nnue = chunk.as_ref().and_then(|c| gpu_backend::pick(&gpu, c));
        let responses = if let Some(nnue) = gpu_nnue {
            // The GPU backend: static evaluation of the whole chunk in one library call.
            let chunk = chunk.take().expect("chunk");
            match gpu_backend::go(nnue, chunk, &tx).await {
                Some(res) => res,
                None => break,
            }
        } else if let Some(chunk) = chunk.take() {
            // Ensure engine process is ready."""),
    ("src/configure.rs", """    #[command(flatten)]
    pub backlog: BacklogOpt,
""", """    /// Evaluate standard-chess analysis on these GPUs (comma-separated device
    /// indices, e.g. 0,1,2,3) with the MI355X NNUE backend instead of engine
    /// processes. Needs a build with the `gpu` feature.
    #[arg(long, global = true)]
    pub gpu_devices: Option<GpuDevices>,

    #[command(flatten)]
    pub backlog: BacklogOpt,
"""),
    ("src/configure.rs", """impl Opt {
    pub fn endpoint(&self) -> Endpoint {""", """/// GPU device indices of the evaluation backend (`--gpu-devices 0,1`).
#[derive(Debug, Clone)]
pub struct GpuDevices(pub Vec<i32>);

impl FromStr for GpuDevices {
    type Err = ParseIntError;

    fn from_str(s: &str) -> Result<GpuDevices, ParseIntError> {
        s.split(',')
            .map(|d| d.trim().parse())
            .collect::<Result<Vec<i32>, _>>()
            .map(GpuDevices)
    }
}

impl Opt {
    pub fn endpoint(&self) -> Endpoint {"""),
    ("src/queue.rs", """    api: ApiStub,
    max_backoff: MaxBackoff,
    logger: Logger,
) -> (QueueStub, QueueActor) {""", """    api: ApiStub,
    max_backoff: MaxBackoff,
    gpu_chunks: bool,
    logger: Logger,
) -> (QueueStub, QueueActor) {"""),
    ("src/queue.rs", """        backlog_opt,
        logger,
        backoff: RandomizedBackoff::new(max_backoff),
    };""", """        backlog_opt,
        logger,
        backoff: RandomizedBackoff::new(max_backoff),
        gpu_chunks,
    };"""),
    ("src/queue.rs", """    backoff: RandomizedBackoff,
    logger: Logger,
}

impl QueueActor {""", """    backoff: RandomizedBackoff,
    logger: Logger,
    gpu_chunks: bool, // the GPU backend takes standard-chess analysis batches whole
}

impl QueueActor {"""),
    ("src/queue.rs", "        match IncomingBatch::from_acquired(self.api.endpoint(), body) {",
     "        match IncomingBatch::from_acquired(self.api.endpoint(), body, self.gpu_chunks) {"),
    ("src/queue.rs", """    fn from_acquired(
        endpoint: &Endpoint,
        body: AcquireResponseBody,
    ) -> Result<IncomingBatch, IncomingError> {""", """    fn from_acquired(
        endpoint: &Endpoint,
        body: AcquireResponseBody,
        gpu_chunks: bool,
    ) -> Result<IncomingBatch, IncomingError> {"""),
    ("src/queue.rs", """                    // Create chunks with overlap.
                    let mut chunks = Vec::new();
                    for prev_and_current_chunked in
                        prev_and_current.chunks(Chunk::MAX_POSITIONS - 1)
                    {""", """                    // The GPU backend takes a standard-chess analysis batch as one chunk:
                    // one library call (the previous-position dummies are evaluated and
                    // dropped like an engine's warm-up positions).
                    let chunk_len = if gpu_chunks && flavor == EngineFlavor::Official {
                        prev_and_current.len().max(1)
                    } else {
                        Chunk::MAX_POSITIONS - 1
                    };

                    // Create chunks with overlap.
                    let mut chunks = Vec::new();
                    for prev_and_current_chunked in prev_and_current.chunks(chunk_len) {"""),
]

PATCHES = [("0001-compile-fixes.patch", STATS), ("0002-gpu-eval-backend.patch", GPU)]


def apply(texts, edits, ref):
    for e in edits:
        path = e[0]
        if path not in texts:
            texts[path] = open(os.path.join(ref, path)).read()
        s = texts[path]
        if e[1] is None:  # replace the span from marker a up to (not including) marker b
            a, b = e[2]
            i = s.index(a)
            j = s.index(b, i)
            texts[path] = s[:i] + e[3] + s[j:]
            continue
        old, new = e[1], e[2]
        if s.count(old) != 1:
            raise SystemExit(f"{path}: edit anchor found {s.count(old)} times: {old[:60]!r}")
        texts[path] = s.replace(old, new)
    return texts


def render(edits, ref):
    texts = apply({}, edits, ref)
    out = []
    for path in sorted(texts):
        orig = open(os.path.join(ref, path)).read().splitlines(keepends=True)
        new = texts[path].splitlines(keepends=True)
        out += difflib.unified_diff(orig, new, "a/" + path, "b/" + path, n=3)
    return "".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    bad = 0
    for name, edits in PATCHES:
        text = render(edits, a.reference)
        p = os.path.join(HERE, name)
        if a.check:
            if not os.path.exists(p) or open(p).read() != text:
                print(f"{name} is not current", file=sys.stderr)
                bad = 1
        else:
            with open(p, "w") as f:
                f.write(text)
    sys.exit(bad)


if __name__ == "__main__":
    main()
