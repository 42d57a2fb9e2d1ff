"""miniraytracer_amd -- MI355X (gfx950) render path for MiniRayTracer scenes.

Host-side mirror of the reference's render interface (the names follow the reference):

* ``ParseArgv(argv)`` / ``MRT_Params``      -- cmdline_parser.cpp:78-107, cmdline_parser.h:5-18
* ``select_scene(scene, aspect)``           -- scene.cpp:25-49 (scenes 0-8, plus 9 = C3 teapot)
* ``Renderer(scene).render(...)``           -- the draw()/draw2() workers over work_queue
                                               (main.cpp:138-243, 347-382), on the GPU
* ``tonemap_argb(img)``                     -- Drago tone map + ARGB32 (main.cpp:416-444)

Everything above the C-ABI is a thin ctypes layer; the render path itself is libmrt.so
(hand-written HIP for gfx950).  No CPU fallback exists.
"""
import ctypes as C
import json
import os

import numpy as np

from . import _lib
from ._lib import MrtError, MrtParams, MrtRenderDesc, MrtSceneView, check, lib

SCENES = ["SCENE_RANDOM_SPHERES", "SCENE_RANDOM_SPHERES_2", "SCENE_TWO_SPHERES", "SCENE_PERLIN_SPHERES",
          "SCENE_EARTH", "SCENE_CORNELL_BOX", "SCENE_CORNELL_SMOKE", "SCENE_BOOK2_FINAL", "SCENE_TRIANGLES",
          "SCENE_TEAPOT_CORNELL"]
MAIN_SEED = 11350390909718046443  # main.cpp:302
ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


def default_params():
    p = MrtParams()
    lib().mrt_default_params(C.byref(p))
    return p


def ParseArgv(argv):
    """Parse reference command-line flags (argv[0] is the program name)."""
    p = MrtParams()
    arr = (C.c_char_p * len(argv))(*[a.encode() for a in argv])
    st = lib().mrt_parse_argv(len(argv), arr, C.byref(p))
    if st != 0:
        raise SystemExit(0)  # -help
    return p


class Scene:
    """Host-side scene built by select_scene (the flattened scene blob)."""

    def __init__(self, handle, scene_id):
        self._h = C.c_void_p(handle)
        self.scene_id = scene_id
        self.view = MrtSceneView()
        check(lib().mrt_scene_blob_view(self._h, C.byref(self.view)), "mrt_scene_blob_view")

    def dump_json(self):
        out = C.c_void_p()
        check(lib().mrt_scene_blob_dump_json(self._h, C.byref(out)), "dump")
        try:
            return json.loads(C.cast(out, C.c_char_p).value.decode())
        finally:
            lib().mrt_free_string(out)

    def worker_seeds(self, n_threads):
        """[(initstate, initseq)] main() gives its worker threads (main.cpp:357-361)."""
        a = np.zeros(n_threads, dtype=np.uint64)
        b = np.zeros(n_threads, dtype=np.uint64)
        check(lib().mrt_worker_seeds(self._h, n_threads, a.ctypes.data, b.ctypes.data), "mrt_worker_seeds")
        return [(int(x), int(y)) for x, y in zip(a, b)]

    def close(self):
        if self._h:
            lib().mrt_scene_blob_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def select_scene(scene, aspect, asset_dir=None):
    h = C.c_void_p()
    ad = (asset_dir or os.environ.get("MRT_ASSET_DIR") or ASSET_DIR).encode()
    check(lib().mrt_select_scene(int(scene), float(aspect), ad, C.byref(h)), f"select_scene({scene})")
    return Scene(h.value, scene)


NUMERICS = ("exact", "fast")


def render_desc(width, height, samples, depth=32, max_luminance=1000.0, mode=0, seed=MAIN_SEED, tile_size=32,
                rank=0, world=1, chunk_samples=0, flags=0, numerics="exact", threads=0, preview=False, ref_order=False,
                pixels=None):
    """Render description; `samples` is floored to a perfect square like main.cpp:319-320.
    numerics: "exact" (bit-for-bit the reference built exact) or "fast" (tolerance contract:
    per-pixel RMSE < 1e-3 vs the reference as shipped; MRT_RF_FAST).  ref_order (CPU backend): the
    reference's own RNG order, one stream per worker thread (Renderer.set_worker_seeds).
    pixels: optional row-major pixel indices to render instead of the rank's tiles (the desc keeps
    a reference to the array; mrt_render_desc.pixels)."""
    if numerics not in NUMERICS:
        raise ValueError(f"numerics must be one of {NUMERICS}")
    if numerics == "fast":
        flags |= _lib.RF_FAST
    if preview:
        flags |= _lib.RF_PREVIEW
    if ref_order:
        flags |= _lib.RF_REF_ORDER
    sq = int(np.sqrt(np.float32(samples)))
    d = MrtRenderDesc(width, height, sq, depth, max_luminance, mode, seed, tile_size, rank, world,
                      chunk_samples, flags, threads)
    if pixels is not None:
        px = np.ascontiguousarray(pixels, dtype=np.uint32)
        d.pixels = px.ctypes.data
        d.n_pixels = px.size
        d._pixels = px  # keeps the list alive as long as the desc
    return d


def local_pixels(desc):
    n = C.c_uint32()
    check(lib().mrt_local_pixels(C.byref(desc), C.byref(n), None), "local_pixels")
    px = np.zeros(n.value, dtype=np.uint32)
    check(lib().mrt_local_pixels(C.byref(desc), C.byref(n), px.ctypes.data), "local_pixels")
    return px


def device_count():
    n = C.c_int()
    st = lib().mrt_init(C.byref(n))
    return n.value if st == 0 else 0


class Renderer:
    """A scene resident in HBM of one device -- or, with device="cpu" (MRT_DEVICE_CPU), held by the
    CPU backend: the same hot-path code compiled for the host, exact numerics contract, worker
    threads over the work_queue tiles (render_desc(threads=...)).  Only an explicit "cpu" selects
    it; without a gfx950 device a GPU Renderer raises."""

    def __init__(self, scene, device=0):
        if device == "cpu":
            device = _lib.DEVICE_CPU
        else:
            n = C.c_int()
            check(lib().mrt_init(C.byref(n)), "mrt_init")
        self.device = device
        self._h = C.c_void_p()
        check(lib().mrt_scene_upload(device, C.byref(scene.view), C.byref(self._h)), "mrt_scene_upload")
        self.scene = scene

    def render(self, desc, cancel=None):
        """Blocking render into a host float32 (H, W, 4) image (row 0 = bottom); returns (img, rays).
        cancel: optional ctypes.c_int; setting it non-zero from another thread stops the render
        (G_isRunning, main.cpp:180/235) and raises MrtError (MRT_ERR_CANCELLED)."""
        img = np.zeros((desc.height, desc.width, 4), dtype=np.float32)
        rays = C.c_uint64()
        check(lib().mrt_render(self._h, C.byref(desc), img.ctypes.data, C.byref(rays), C.byref(cancel) if cancel is not None else None),
              "mrt_render")
        return img, rays.value

    def set_worker_seeds(self, seeds):
        """CPU backend: the (initstate, initseq) of each worker thread (main.cpp:357-366, e.g.
        scene.worker_seeds(n)) for renders in the reference's RNG order (render_desc(ref_order=True))."""
        a = np.array([s[0] for s in seeds], dtype=np.uint64)
        b = np.array([s[1] for s in seeds], dtype=np.uint64)
        check(lib().mrt_set_worker_seeds(self._h, len(seeds), a.ctypes.data, b.ctypes.data), "mrt_set_worker_seeds")

    def prepare(self, desc):
        check(lib().mrt_prepare(self._h, C.byref(desc)), "mrt_prepare")

    def render_device(self, desc, d_out_ptr, d_rays_ptr, stream_ptr=0):
        """Enqueue a render into device memory (torch tensor data_ptr()s) on a HIP stream."""
        check(lib().mrt_render_device(self._h, C.byref(desc), C.c_void_p(d_out_ptr), C.c_void_p(d_rays_ptr),
                                      C.c_void_p(stream_ptr)), "mrt_render_device")

    def join(self, stream_ptr=0):
        """Order a HIP stream after this context's last render_device (its fold runs on the context's
        own stream under RF_FOLD_ASYNC): the worker threads' join() (main.cpp:490-493)."""
        check(lib().mrt_render_join(self._h, C.c_void_p(stream_ptr)), "mrt_render_join")

    def preview(self, width, height):
        """The running render as the reference's UI thread sees G_linearBackBuffer (main.cpp:387-444):
        (H, W, 4) float32 image after `samples` samples of every pixel, callable from another thread
        while render() runs.  GPU: renders made with flags=RF_PREVIEW (render_desc(preview=True))."""
        img = np.zeros((height, width, 4), dtype=np.float32)
        n = C.c_uint32()
        check(lib().mrt_preview(self._h, img.ctypes.data, C.byref(n)), "mrt_preview")
        return img, n.value

    def progress(self):
        """Percent of the current / last render's paths handed out (work_queue::getPercentDone)."""
        pct = C.c_float()
        check(lib().mrt_progress(self._h, C.byref(pct)), "mrt_progress")
        return pct.value

    def kernel_info(self):
        """dict(features, kernel_features, lds_bytes, grid, prog_ops) of the path kernel this scene runs."""
        ki = _lib.KernelInfo()
        check(lib().mrt_scene_kernel_info(self._h, C.byref(ki)), "mrt_scene_kernel_info")
        return {k: getattr(ki, k) for k, _ in ki._fields_}

    def kernel_ms(self):
        """(total ms, launches) of the path kernel in the last render (HIP events on its stream)."""
        ms, n = C.c_float(), C.c_uint32()
        check(lib().mrt_kernel_ms(self._h, C.byref(ms), C.byref(n)), "mrt_kernel_ms")
        return ms.value, n.value

    def paths(self, n_paths):
        """Per-path radiance and ray counts of the last MRT_RF_PATH_DEBUG render ([s][local pixel])."""
        rgb = np.zeros((n_paths, 3), dtype=np.float32)
        rays = np.zeros(n_paths, dtype=np.uint32)
        check(lib().mrt_render_debug(self._h, rgb.ctypes.data, rays.ctypes.data, n_paths), "mrt_render_debug")
        return rgb, rays

    def close(self):
        if self._h:
            lib().mrt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    """ncclGetUniqueId for mrt_comm_init_rank (rank 0 makes it, the others receive it out of band)."""
    buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
    check(lib().mrt_comm_unique_id(buf), "mrt_comm_unique_id")
    return bytes(buf)


def gather_shard_pixels(desc):
    """Pixels of the largest rank shard of desc's tile deal (the RCCL gather's padded shard)."""
    n = C.c_uint32()
    check(lib().mrt_gather_shard_pixels(C.byref(desc), C.byref(n)), "mrt_gather_shard_pixels")
    return n.value


class Comm:
    """One rank of an RCCL communicator for the framebuffer gather (include/mrt.h "multi-GPU"):
    Comm(device, world, rank, uid) per process (mrt_comm_init_rank), or Comm.init_all(devices) for one
    process driving every GPU (mrt_comm_init_all)."""

    def __init__(self, device=0, world=1, rank=0, uid=None, _handle=None):
        self.device, self.world, self.rank = device, world, rank
        self._h = C.c_void_p(_handle)
        if _handle is None:
            buf = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid if uid is not None else comm_unique_id())
            check(lib().mrt_comm_init_rank(device, world, rank, buf, C.byref(self._h)), "mrt_comm_init_rank")

    @classmethod
    def init_all(cls, devices):
        n = len(devices)
        devs = (C.c_int * n)(*devices)
        hs = (C.c_void_p * n)()
        check(lib().mrt_comm_init_all(n, devs, hs), "mrt_comm_init_all")
        return [cls(devices[r], n, r, _handle=hs[r]) for r in range(n)]

    def gather_frame(self, desc, d_local_ptr, d_frame_ptr, d_rays_ptr=0, stream_ptr=0):
        """Collective: this rank's shard (render_device output) to the root's W*H float4 frame, rays
        all-reduced in place (device pointers, e.g. torch data_ptr()s; enqueued on a HIP stream)."""
        check(lib().mrt_gather_frame(self._h, C.byref(desc), C.c_void_p(d_local_ptr), C.c_void_p(d_frame_ptr or None),
                                     C.c_void_p(d_rays_ptr or None), C.c_void_p(stream_ptr)), "mrt_gather_frame")

    def render_gather(self, renderer, desc):
        """Collective render + RCCL gather: the whole (H, W, 4) image on the root (None elsewhere) and
        the ray total of all ranks."""
        img = np.zeros((desc.height, desc.width, 4), dtype=np.float32) if self.rank == 0 else None
        rays = C.c_uint64()
        check(lib().mrt_render_gather(renderer._h, self._h, C.byref(desc), img.ctypes.data if img is not None else None,
                                      C.byref(rays)), "mrt_render_gather")
        return img, rays.value

    def close(self):
        if self._h:
            lib().mrt_comm_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def tonemap_device(d_rgb_ptr, n, d_lwmax_ptr, d_argb_ptr, stream_ptr=0, reduce=True):
    """Device tone map of n float4 pixels (torch data_ptr()s).  reduce=True first max-reduces the
    luminance into *d_lwmax (which the caller zeroed); pass reduce=False after combining L_wmax
    across ranks yourself."""
    if reduce:
        check(lib().mrt_lum_max_device(C.c_void_p(d_rgb_ptr), n, C.c_void_p(d_lwmax_ptr), C.c_void_p(stream_ptr)), "mrt_lum_max_device")
    check(lib().mrt_tonemap_device(C.c_void_p(d_rgb_ptr), n, C.c_void_p(d_lwmax_ptr), C.c_void_p(d_argb_ptr), C.c_void_p(stream_ptr)),
          "mrt_tonemap_device")


def tonemap_argb(img):
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape[:2]
    out = np.zeros((h, w), dtype=np.uint32)
    check(lib().mrt_tonemap_argb(img.ctypes.data, w, h, out.ctypes.data), "tonemap")
    return out


def write_pfm(path, img):
    """Linear PFM, rows bottom-to-top (the PFM convention == G_linearBackBuffer order)."""
    h, w = img.shape[:2]
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(img[..., :3], dtype="<f4").tobytes())


def read_pfm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], dtype="<f4").reshape(h, w, 3)


def write_ppm(path, argb):
    """Tone-mapped 8-bit PPM, displayed top row first (SDL_FLIP_VERTICAL, platform_linux.cpp:84)."""
    h, w = argb.shape
    rgb = np.stack([(argb >> 16) & 255, (argb >> 8) & 255, argb & 255], axis=-1).astype(np.uint8)[::-1]
    with open(path, "wb") as f:
        f.write(f"P6\n{w} {h}\n255\n".encode())
        f.write(rgb.tobytes())
