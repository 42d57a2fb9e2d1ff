"""Host-side surface (CPU only): the C-ABI library loads and exports every declared symbol, the
reference's flags parse the same way, work_queue tile order, per-rank ownership, tone map."""
import ctypes
import json
import os
import re
import types

import numpy as np

from conftest import GOLDEN
import pytest

from conftest import ROOT


def declared_symbols():
    names = set()
    for h in ("mrt.h",):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(mrt_[a-z_0-9]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol(mrt):
    lib = ctypes.CDLL(mrt._lib.LIB_PATH)
    decl = declared_symbols()
    assert len(decl) >= 20
    missing = [n for n in sorted(decl) if not hasattr(lib, n)]
    assert not missing, missing
    assert set(mrt._lib.EXPORTS) <= decl


def test_abi_version_and_unknown_flags(mrt):
    """ABI 6: the binding checks mrt_abi_version() at load; MRT_RF_FOLD_ASYNC moved to
    0x40, and the bit it used to share with the removed MRT_RF_SPLIT (0x20), like every unknown bit,
    is refused with MRT_ERR_INVALID by every entry point that reads a desc, instead of silently
    meaning something else.  The RCCL gather's padded shard is the largest rank's pixel count."""
    assert mrt.lib().mrt_abi_version() == mrt._lib.ABI_VERSION == 6
    assert mrt._lib.RF_FOLD_ASYNC == 0x40
    for bad in (0x20, 0x80, 1 << 31):
        with pytest.raises(mrt.MrtError, match="0x20" if bad == 0x20 else "unknown flag"):
            mrt.local_pixels(mrt.render_desc(64, 48, 4, flags=bad))
    with pytest.raises(mrt.MrtError, match="0x20"):
        mrt.Renderer(mrt.select_scene(5, 1.0), "cpu").render(mrt.render_desc(16, 16, 1, flags=0x20))
    for world in (1, 3, 8):
        counts = [len(mrt.local_pixels(mrt.render_desc(200, 100, 4, tile_size=16, rank=r, world=world))) for r in range(world)]
        assert sum(counts) == 200 * 100
        assert mrt.gather_shard_pixels(mrt.render_desc(200, 100, 4, tile_size=16, world=world)) == max(counts)


def test_oracle_is_not_linked_into_the_product(mrt):
    # the product .so never references the oracle (test infrastructure only)
    data = open(mrt._lib.LIB_PATH, "rb").read()
    assert b"oracle_" not in data and b"liboracle" not in data


def test_parse_argv_matches_reference_defaults_and_ranges(mrt):
    p = mrt.ParseArgv(["mrt"])  # MRT_Params defaults (cmdline_parser.h:5-18)
    assert (p.buffer_width, p.buffer_height, p.samples_per_pixel, p.tile_size, p.num_threads, p.max_bounces,
            p.scene_select, p.threading_mode) == (500, 500, 128, 32, 0, 32, 8, 1)
    assert p.max_luminance == 1000.0 and p.seed == mrt.MAIN_SEED
    p = mrt.ParseArgv(["mrt", "-scene", "5", "-width", "640", "-height", "0x1e0", "-samples", "1024", "-depth", "8",
                       "-mode", "0", "-maxlum", "50.5", "-tilesize", "16"])
    assert (p.scene_select, p.buffer_width, p.buffer_height, p.samples_per_pixel, p.max_bounces, p.threading_mode,
            p.tile_size) == (5, 640, 480, 1024, 8, 0, 16)
    assert p.max_luminance == np.float32(50.5)
    # out-of-range values are ignored with a warning (ReadParameter, cmdline_parser.cpp:51-54)
    p = mrt.ParseArgv(["mrt", "-scene", "12", "-mode", "2", "-width", "0", "-depth"])
    assert (p.scene_select, p.threading_mode, p.buffer_width, p.max_bounces) == (8, 1, 500, 32)
    # -threads keeps the reference's meaning (CPU worker threads); GPUs and numerics have their own flags
    p = mrt.ParseArgv(["mrt", "-threads", "3", "-gpus", "2", "-numerics", "exact"])
    assert (p.num_threads, p.gpus, p.numerics) == (3, 2, 0)
    p = mrt.ParseArgv(["mrt", "-numerics", "bogus"])
    assert (p.num_threads, p.gpus, p.numerics) == (0, 0, 1)


def test_default_render_desc_carries_numerics(mrt):
    for num, flag in ((0, 0), (1, mrt._lib.RF_FAST)):
        p = mrt.ParseArgv(["mrt", "-scene", "5", "-samples", "17", "-numerics", str(num)])
        d = mrt._lib.MrtRenderDesc()
        mrt.lib().mrt_default_render_desc(ctypes.byref(p), ctypes.byref(d))
        assert (d.sqrt_samples, d.flags & mrt._lib.RF_FAST) == (4, flag)


def test_order_flag_defaults(mrt):
    """-order: the reference's RNG order is the CPU backend's default (its -threads 1 run is then
    reproducible), per-path keys the GPU's; -order path / ref override; the desc carries it."""
    cases = [(["-backend", "cpu"], 1), ([], 0), (["-backend", "cpu", "-order", "path"], 0), (["-order", "ref"], 1)]
    for args, order in cases:
        p = mrt.ParseArgv(["mrt"] + args)
        assert p.order == order, args
        d = mrt._lib.MrtRenderDesc()
        mrt.lib().mrt_default_render_desc(ctypes.byref(p), ctypes.byref(d))
        assert bool(d.flags & mrt._lib.RF_REF_ORDER) == bool(order)


def test_render_flags_match_header(mrt):
    """The ctypes mirror's MRT_RF_* bits are the header's (include/mrt.h)."""
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "mrt.h")).read()
    bits = {m.group(1): int(m.group(2), 16) for m in re.finditer(r"#define MRT_RF_(\w+) (0x[0-9a-fA-F]+)u", hdr)}
    assert set(bits) == {"PATH_DEBUG", "FAST", "PREVIEW", "FOLD_BEHIND", "FOLD_ASYNC", "REF_ORDER"}
    for name, v in bits.items():
        assert getattr(mrt._lib, "RF_" + name) == v, name


def header_struct(name):
    """(field, C type) of `typedef struct <name> {...} <name>;` in include/mrt.h, comments dropped."""
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "mrt.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), hdr, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    out = []
    for decl in body.split(";"):
        decl = " ".join(decl.split())
        if not decl:
            continue
        m = re.match(r"(const )?(uint32_t|uint64_t|float)(\s*\*)?\s+(.*)", decl)
        ctype = "ptr" if m.group(3) else m.group(2)
        out += [(n.strip(), ctype) for n in m.group(4).split(",")]
    return out


@pytest.mark.parametrize("cname,pyname", [("mrt_render_desc", "MrtRenderDesc"), ("mrt_params", "MrtParams")])
def test_abi_structs_match_header(mrt, cname, pyname):
    """The ctypes mirrors of the C-ABI's argument structs have the header's fields, in order, with
    the same types (a field added on one side only would shift every later one)."""
    want = {"uint32_t": ctypes.c_uint32, "uint64_t": ctypes.c_uint64, "float": ctypes.c_float, "ptr": ctypes.c_void_p}
    fields = getattr(mrt._lib, pyname)._fields_
    assert [f for f, _ in fields] == [n for n, _ in header_struct(cname)]
    for (f, t), (_, ct) in zip(fields, header_struct(cname)):
        assert t is want[ct], f


def test_kernel_info_layout_matches_header(mrt):
    """The ctypes mirror of mrt_kernel_info has the header's fields, in order, with the same types:
    a field added on one side only would shift every later one."""
    want = {"uint32_t": ctypes.c_uint32, "uint64_t": ctypes.c_uint64}
    hdr = header_struct("mrt_kernel_info")
    assert [f for f, _ in mrt._lib.KernelInfo._fields_] == [n for n, _ in hdr]
    for (f, t), (_, ct) in zip(mrt._lib.KernelInfo._fields_, hdr):
        assert t is want[ct], f


def reference_tiles(W, H, ts):
    """work_queue::work_queue (work_queue.cpp:64-128), restated in numpy-free Python."""
    xc, yc = (W + ts - 1) // ts, (H + ts - 1) // ts
    tiles = [(x * ts, min(x * ts + ts, W), y * ts, min(y * ts + ts, H)) for y in range(yc) for x in range(xc)]
    m = max(xc, yc)
    po2 = 1
    while po2 < m:
        po2 *= 2
    log2 = po2.bit_length() - 1

    def d2xy(n, d):
        x = y = 0
        s, t = 1, d
        while s < n:
            rx = 1 & (t // 2)
            ry = 1 & (t ^ rx)
            if ry == 0:
                if rx == 1:
                    x, y = s - 1 - x, s - 1 - y
                x, y = y, x
            x += s * rx
            y += s * ry
            t //= 4
            s *= 2
        return x, y

    def rev(v, bits):
        return int(format(v, "032b")[::-1], 2) >> (32 - bits) if bits else 0

    out = []
    for d in range(po2 * po2):
        x, y = d2xy(po2, d)
        x, y = rev(x, log2), rev(y, log2)
        if x < xc and y < yc:
            out.append(tiles[x + y * xc])
        if len(out) == len(tiles):
            break
    return out


M64 = (1 << 64) - 1


def tile_owners(n, world):
    """The multi-GPU deal (mrt_common.cpp mrt_internal_tile_owners): rounds of `world` consecutive
    work_queue tiles, round b to the ranks in the order of a Fisher-Yates permutation whose draws
    are splitmix64 iterated from b."""
    def mix(z):
        z = (z + 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)
    own = [0] * n
    if world <= 1:
        return own
    for b in range((n + world - 1) // world):
        perm, st = list(range(world)), b
        for i in range(world - 1, 0, -1):
            st = mix(st)
            j = st % (i + 1)
            perm[i], perm[j] = perm[j], perm[i]
        for j in range(world):
            if b * world + j < n:
                own[b * world + j] = perm[j]
    return own


def test_tile_deal_is_balanced_and_permuted():
    """Every round of `world` tiles gives each rank exactly one tile, and not always the same one."""
    own = tile_owners(4096, 8)
    for b in range(512):
        assert sorted(own[8 * b:8 * b + 8]) == list(range(8))
    assert any(own[8 * b:8 * b + 8] != own[:8] for b in range(1, 512))


@pytest.mark.parametrize("W,H,ts,world", [(500, 500, 32, 1), (500, 500, 32, 8), (200, 100, 32, 3), (37, 23, 7, 2),
                                           (1, 1, 32, 1), (1024, 1024, 32, 8), (64, 640, 16, 5), (500, 500, 4, 8)])
def test_local_pixels_follow_work_queue_tiles(mrt, W, H, ts, world):
    tiles = reference_tiles(W, H, ts)
    own = tile_owners(len(tiles), world)
    seen = np.zeros(W * H, dtype=np.int32)
    for rank in range(world):
        px = mrt.local_pixels(mrt.render_desc(W, H, 16, tile_size=ts, rank=rank, world=world))
        exp = [x + y * W for k, (x0, x1, y0, y1) in enumerate(tiles) if own[k] == rank
               for y in range(y0, y1) for x in range(x0, x1)]
        assert px.tolist() == exp
        seen[px] += 1
    assert np.all(seen == 1)


@pytest.mark.parametrize("sid", [5, 2])
def test_tonemap_matches_reference_display_loop(mrt, sid):
    """Drago mapping (main.cpp:416-444) + ARGB32 (vec3.h:327-333): the host tone map equals, bit for
    bit, the G_backBuffer the reference's own display loop produced from the same linear buffer
    (tests/golden/tonemap_<id>.npz, exact reference build)."""
    g = np.load(os.path.join(GOLDEN, f"tonemap_{sid}.npz"))
    h, w = g["argb"].shape
    img = np.zeros((h, w, 4), dtype=np.float32)
    img[..., :3] = g["linear"]
    argb = mrt.tonemap_argb(img)
    assert np.array_equal(argb, g["argb"]), np.argwhere(argb != g["argb"])[:5]


def test_tonemap_formula_with_libm(mrt):
    """The same mapping restated with numpy's libm logs/pow: equal up to one level per channel
    (the numerics contract's log/pow may differ from libm in the last float bit)."""
    rng = np.random.default_rng(0)
    img = np.zeros((7, 9, 4), dtype=np.float32)
    img[..., :3] = rng.exponential(0.5, size=(7, 9, 3)).astype(np.float32)
    img[3, 4, :3] = 40.0
    argb = mrt.tonemap_argb(img)
    f = np.float32
    lum = (img[..., 0] * f(0.212655) + img[..., 1] * f(0.715158)) + img[..., 2] * f(0.072187)
    lwmax = lum.max()
    invlogmax = f(1) / f(np.log10(np.float64(lwmax + f(1))))
    bias = f(np.log(np.float64(f(0.7)))) / f(np.log(np.float64(f(0.5))))
    for y in range(7):
        for x in range(9):
            l = lum[y, x]
            loglw = f(np.log(np.float64(l + f(1))))
            pw = f(np.power(np.float64(l * (f(1) / lwmax)), np.float64(bias)))
            ln = (f(230.0) * f(0.01) * invlogmax) * (loglw / f(np.log(np.float64(f(2) + pw * f(8)))))
            c = [(ln * img[y, x, k]) / (l + f(0.00001)) for k in range(3)]
            c = [int(f(min(v, f(1))) * f(255.99)) for v in c]
            got = [(int(argb[y, x]) >> s) & 255 for s in (16, 8, 0)]
            assert all(abs(a - b) <= 1 for a, b in zip(got, c))


def test_select_scene_errors_are_loud(mrt, tmp_path):
    with pytest.raises(mrt.MrtError):
        mrt.select_scene(8, 1.0, asset_dir=str(tmp_path))  # no bunny asset -> MRT_ERR_IO
    with pytest.raises(mrt.MrtError):
        mrt.select_scene(11, 1.0)


def test_packed_mesh_equals_obj_parse(mrt, tmp_path):
    """assets/*.mesh hold exactly the records the OBJ parser produces (checked where the OBJ exists)."""
    obj = "/root/reference/obj/bunny.obj"
    if not os.path.exists(obj):
        pytest.skip("reference OBJ not present on this host")
    out = tmp_path / "bunny.mesh"
    assert mrt.lib().mrt_pack_obj(obj.encode(), str(out).encode()) == 0
    assert out.read_bytes() == open(os.path.join(ROOT, "assets", "bunny.mesh"), "rb").read()


def test_bench_roofline_prices_pmc_per_ray(tmp_path):
    """bench.py's roofline: VALU issue rate of the launch from the committed per-ray PMC figures and
    the live kernel time, frac against 1024 SIMDs x 2.4 GHz / 2; a rank's share priced by its own
    rays (world > 1); a PMC file of another workload is not used."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    pmc = tmp_path / "p.json"
    pmc.write_text(json.dumps({"config": [5, 500, 500, 1024, 32], "source": "x",
                               "by_numerics": {"fast": {"valu_insts_per_ray": 9.0, "hbm_bytes_per_ray": 7.0, "valu_lane_util": 0.6,
                                                        "valu_busy": 0.7}}}))
    args = types.SimpleNamespace(scene=5, width=500, height=500, depth=32, pmc_json=str(pmc))
    ki = dict(grid=1, wg=64, lds_bytes=0, vgprs=72, tree_nodes=0, kernel_features=0x2000 | 0x800 | 0x8 | (1 << 16), build=2)
    r = bench.roofline(args, 8.0, 778e6, "fast", ki)
    assert r["bound"] == "valu" and r["peak"] == pytest.approx(1228.8)
    # the kernel's rocprofv3 name from the build the library reports (mrt_kernel_info.build)
    assert r["kernel"] == "mrt_path_kernel_fastz"
    assert bench.roofline(args, 8.0, 778e6, "fast", dict(ki, build=1))["kernel"] == "mrt_path_kernel_fast"
    assert bench.roofline(args, 8.0, 778e6, "fast", dict(ki, build=3))["kernel"] == "mrt_path_kernel_pex"
    assert bench.roofline(args, 8.0, 778e6, "exact", dict(ki, build=0))["kernel"] == "mrt_path_kernel"
    assert r["achieved"] == pytest.approx(9.0 * 778e6 / 8e-3 / 1e9, rel=1e-3)
    assert 0 < r["frac"] <= 1 and r["traffic"] == round(7.0 * 778e6)
    half = bench.roofline(args, 4.0, 389e6, "fast", ki)  # a rank's half: same rates
    assert half["frac"] == pytest.approx(r["frac"], rel=1e-3) and half["hbm_frac"] == pytest.approx(r["hbm_frac"], rel=1e-3)
    args.width = 640
    assert bench.roofline(args, 8.0, 778e6, "fast", ki)["frac"] is None


def _lin_program(mrt, sid, rewritten):
    import ctypes as C
    sc = mrt.select_scene(sid, 1.0)
    fn = mrt.lib().mrt_debug_lin_program
    fn.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
    fn.restype = C.c_int
    codes = np.zeros(4096, dtype=np.uint32)
    skips = np.zeros(4096, dtype=np.uint32)
    n = np.zeros(1, dtype=np.uint32)
    assert fn(C.byref(sc.view), int(rewritten), codes.ctypes.data, skips.ctypes.data, 4096, n.ctypes.data) == 0
    sc.close()
    return codes[:int(n[0])], skips[:int(n[0])]


@pytest.mark.parametrize("sid", [5, 8, 9, 0, 7])
def test_program_rewrite_structure(mrt, sid):
    """The tolerance contract's program rewrite (mrt_sig.h lin_rewrite_fast): the Cornell rooms'
    inward-facing walls become one LOP_ROOM + LOP_ROOMDATA pair, an instance of one box.h list is
    flagged MRT_F_BOXINST, the root object_list's LIST / LIST_END pair is dropped, the op after
    which the walk reaches END is flagged MRT_F_LAST (exactly one), nothing else changes, and every
    LIST / INST skip still lands on its END op.  Scenes without rooms (0, 7) keep
    their program but for the root pair."""
    LIST, LIST_END, INST, INST_END, ROOM, ROOMDATA, END = 3, 4, 5, 6, 10, 11, 0
    c0, s0 = _lin_program(mrt, sid, False)
    c1, s1 = _lin_program(mrt, sid, True)
    op0, op1 = c0 & 0xFF, c1 & 0xFF
    assert ROOM not in op0 and ROOMDATA not in op0
    root = bool(op0[0] == LIST and s0[0] == len(op0) - 2 and op0[-2] == LIST_END and op0[-1] == END)
    assert root == (sid != 0)  # (an object_list at the root; scene 0 is a bvh_node)
    rooms = int((op1 == ROOM).sum())
    if sid in (5, 8, 9):
        assert rooms == 1 and op1[list(op1).index(ROOM) + 1] == ROOMDATA
        # the room's walls (five rects in these scenes) replaced by the pair, the root pair gone
        assert len(op1) == len(op0) - 5 + 2 - 2
    else:
        kept = np.concatenate([c0[1:-2], c0[-1:]]) if root else c0
        assert rooms == 0 and np.array_equal(kept & ~np.uint32(0x60 << 16), c1 & ~np.uint32(0x60 << 16))
    assert int(((c1 >> 16) & 0x40 != 0).sum()) == 1 and not ((c0 >> 16) & 0x40).any()
    boxinst = [(c >> 16) & 0x20 for c, o in zip(c1, op1) if o == INST]
    assert sum(1 for b in boxinst if b) == (1 if sid == 5 else 0)
    for i, (o, k) in enumerate(zip(op1, s1)):
        if o in (LIST, INST):
            assert i < k < len(op1) and op1[k] == (LIST_END if o == LIST else INST_END), (i, o, k)


def test_volume_boundary_subprogram_structure(mrt):
    """Cornell smoke (scene 6, scene.cpp:334-376): each constant_volume bounded by
    translate(rotate_y(box)) compiles to a LOP_VOLUME op flagged MRT_F_VSUB whose skip lands just past
    its boundary sub-program -- the fused instance, box.h's list of six rects, their END ops -- so the
    main walk steps over it and the volume op walks it twice per query (mrt_lin.h lin_sub_t)."""
    PRIM, LIST, LIST_END, INST, INST_END, VOLUME, VSUB = 1, 3, 4, 5, 6, 8, 0x80
    c, s = _lin_program(mrt, 6, False)
    op = c & 0xFF
    vols = [i for i, o in enumerate(op) if o == VOLUME]
    assert len(vols) == 2
    for i in vols:
        assert (c[i] >> 16) & VSUB
        body = list(op[i + 1:s[i]])
        assert body == [INST, LIST] + [PRIM] * 6 + [LIST_END, INST_END], body
        assert s[i + 1] == s[i] - 1 and s[i + 2] == s[i] - 2  # the instance's and the list's END ops
    # book2's volumes keep their primitive boundary (LOP_VBOUND after the op, no flag)
    c7, _ = _lin_program(mrt, 7, False)
    v7 = [i for i, o in enumerate(c7 & 0xFF) if o == VOLUME]
    assert v7 and all(not ((c7[i] >> 16) & VSUB) and (c7[i + 1] & 0xFF) == 9 for i in v7)
