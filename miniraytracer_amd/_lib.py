"""ctypes binding of the C-ABI in include/mrt.h (miniraytracer_amd/libmrt.so).

The library is built in-tree by ``make`` (``__graft_entry__.build()``).  There is no Python or CPU
fallback for the render path: if libmrt.so is missing or fails to load, importing the render API
raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmrt.so")
# experiment hook (tools/ab.sh): load an A/B build from exp/ instead of the in-tree library
if os.environ.get("MRT_EXPERIMENT_LIB"):
    LIB_PATH = os.path.abspath(os.environ["MRT_EXPERIMENT_LIB"])

MRT_NONE = 0xFFFFFFFF
RF_PATH_DEBUG = 0x1
RF_FAST = 0x2  # tolerance numerics contract (include/mrt.h MRT_RF_FAST)
RF_PREVIEW = 0x4  # keep a progressive preview for mrt_preview (include/mrt.h MRT_RF_PREVIEW)
RF_FOLD_BEHIND = 0x8  # mode-0 fold that runs beside another context's path kernel (include/mrt.h)
RF_FOLD_ASYNC = 0x40  # the fold beside the next render's path kernel, on the context's own stream (include/mrt.h; ABI 6)
RF_REF_ORDER = 0x10  # CPU backend: the reference's own RNG order (worker streams, work_queue order)
DEVICE_CPU = -1  # mrt_scene_upload device of the CPU backend (include/mrt.h MRT_DEVICE_CPU)
ABI_VERSION = 6  # include/mrt.h MRT_ABI_VERSION: checked against mrt_abi_version() at load
COMM_ID_BYTES = 128  # include/mrt.h MRT_COMM_ID_BYTES


class MrtParams(C.Structure):
    """MRT_Params (cmdline_parser.h:5-18) + seed."""
    _fields_ = [("window_width", C.c_uint32), ("window_height", C.c_uint32),
                ("buffer_width", C.c_uint32), ("buffer_height", C.c_uint32),
                ("samples_per_pixel", C.c_uint32), ("tile_size", C.c_uint32),
                ("num_threads", C.c_uint32), ("max_bounces", C.c_uint32),
                ("scene_select", C.c_uint32), ("threading_mode", C.c_uint32),
                ("max_luminance", C.c_float), ("delay", C.c_uint32), ("seed", C.c_uint64),
                ("gpus", C.c_uint32), ("numerics", C.c_uint32), ("backend", C.c_uint32), ("order", C.c_uint32)]


class MrtRenderDesc(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("sqrt_samples", C.c_uint32),
                ("max_bounces", C.c_uint32), ("max_luminance", C.c_float), ("mode", C.c_uint32),
                ("seed", C.c_uint64), ("tile_size", C.c_uint32), ("rank", C.c_uint32),
                ("world", C.c_uint32), ("chunk_samples", C.c_uint32), ("flags", C.c_uint32),
                ("threads", C.c_uint32), ("pixels", C.c_void_p), ("n_pixels", C.c_uint32)]


class MrtCamera(C.Structure):
    _fields_ = [(n, C.c_float * 4) for n in ("origin", "u", "v", "w", "llcorner", "horz", "vert")] + \
               [("lens_radius", C.c_float), ("time0", C.c_float), ("time1", C.c_float), ("pad", C.c_float)]


class MrtSceneView(C.Structure):
    _fields_ = [("scene_id", C.c_uint32), ("root", C.c_uint32), ("biased", C.c_uint32), ("sky", C.c_uint32),
                ("camera", MrtCamera),
                ("nodes", C.c_void_p), ("n_nodes", C.c_uint32),
                ("children", C.c_void_p), ("n_children", C.c_uint32),
                ("mesh_nodes", C.c_void_p), ("n_mesh_nodes", C.c_uint32),
                ("tri_geo", C.c_void_p), ("tri_nrm", C.c_void_p), ("n_tris", C.c_uint32),
                ("materials", C.c_void_p), ("n_materials", C.c_uint32),
                ("textures", C.c_void_p), ("n_textures", C.c_uint32),
                ("perlin_ranvec", C.c_void_p), ("perlin_perm", C.c_void_p),
                ("texels", C.c_void_p), ("n_texels", C.c_uint64)]


class KernelInfo(C.Structure):
    _fields_ = [("features", C.c_uint32), ("kernel_features", C.c_uint32), ("lds_bytes", C.c_uint32),
                ("grid", C.c_uint32), ("prog_ops", C.c_uint32), ("vgprs", C.c_uint32), ("wg", C.c_uint32),
                ("tree_nodes", C.c_uint32), ("build", C.c_uint32), ("pad", C.c_uint32),
                ("handed_over", C.c_uint64), ("handover_lost", C.c_uint64)]
BUILDS = ("exact", "fast", "fastz", "pex")  # MRT_BUILD_*: the kernel build (mrt_path_kernel[_fast|_fastz|_pex])


FT_LIN = 1 << 11  # kernel feature bit: linear hit program (mrt_lin.h)
FT_VSUB = 1 << 14  # kernel feature bit: volumes bounded by sub-programs (mrt_lin.h lin_sub_t; Cornell smoke)


class MrtError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libmrt.so (fails loudly when it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MrtError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    st = C.c_int
    L.mrt_abi_version.restype = C.c_uint32
    if L.mrt_abi_version() != ABI_VERSION:
        raise MrtError(f"{LIB_PATH}: ABI {L.mrt_abi_version()}, this binding is ABI {ABI_VERSION}: rebuild (make)")
    L.mrt_default_params.argtypes = [C.POINTER(MrtParams)]
    L.mrt_parse_argv.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(MrtParams)]
    L.mrt_parse_argv.restype = st
    L.mrt_select_scene.argtypes = [C.c_uint32, C.c_float, C.c_char_p, C.POINTER(C.c_void_p)]
    L.mrt_select_scene.restype = st
    L.mrt_scene_blob_view.argtypes = [C.c_void_p, C.POINTER(MrtSceneView)]
    L.mrt_scene_blob_view.restype = st
    L.mrt_scene_blob_dump_json.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    L.mrt_scene_blob_dump_json.restype = st
    L.mrt_free_string.argtypes = [C.c_void_p]
    L.mrt_scene_blob_free.argtypes = [C.c_void_p]
    L.mrt_init.argtypes = [C.POINTER(C.c_int)]
    L.mrt_init.restype = st
    L.mrt_scene_upload.argtypes = [C.c_int, C.POINTER(MrtSceneView), C.POINTER(C.c_void_p)]
    L.mrt_scene_upload.restype = st
    L.mrt_scene_free.argtypes = [C.c_void_p]
    L.mrt_default_render_desc.argtypes = [C.POINTER(MrtParams), C.POINTER(MrtRenderDesc)]
    L.mrt_local_pixels.argtypes = [C.POINTER(MrtRenderDesc), C.POINTER(C.c_uint32), C.c_void_p]
    L.mrt_local_pixels.restype = st
    L.mrt_render.argtypes = [C.c_void_p, C.POINTER(MrtRenderDesc), C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p]
    L.mrt_render.restype = st
    L.mrt_render_device.argtypes = [C.c_void_p, C.POINTER(MrtRenderDesc), C.c_void_p, C.c_void_p, C.c_void_p]
    L.mrt_render_device.restype = st
    L.mrt_render_join.argtypes = [C.c_void_p, C.c_void_p]
    L.mrt_render_join.restype = st
    L.mrt_prepare.argtypes = [C.c_void_p, C.POINTER(MrtRenderDesc)]
    L.mrt_prepare.restype = st
    L.mrt_render_debug.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    L.mrt_render_debug.restype = st
    L.mrt_progress.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
    L.mrt_progress.restype = st
    L.mrt_lum_max_device.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    L.mrt_lum_max_device.restype = st
    L.mrt_tonemap_device.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
    L.mrt_tonemap_device.restype = st
    L.mrt_preview.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32)]
    L.mrt_preview.restype = st
    L.mrt_scene_kernel_info.argtypes = [C.c_void_p, C.POINTER(KernelInfo)]
    L.mrt_scene_kernel_info.restype = st
    L.mrt_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_uint32)]
    L.mrt_kernel_ms.restype = st
    L.mrt_worker_seeds.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    L.mrt_worker_seeds.restype = st
    L.mrt_set_worker_seeds.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    L.mrt_set_worker_seeds.restype = st
    L.mrt_pack_obj.argtypes = [C.c_char_p, C.c_char_p]
    L.mrt_pack_obj.restype = st
    L.mrt_tonemap_argb.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.mrt_tonemap_argb.restype = st
    L.mrt_strerror.argtypes = [C.c_int]
    L.mrt_strerror.restype = C.c_char_p
    L.mrt_last_error.restype = C.c_char_p
    L.mrt_comm_unique_id.argtypes = [C.c_void_p]
    L.mrt_comm_unique_id.restype = st
    L.mrt_comm_init_rank.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_void_p, C.POINTER(C.c_void_p)]
    L.mrt_comm_init_rank.restype = st
    L.mrt_comm_init_all.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p]
    L.mrt_comm_init_all.restype = st
    L.mrt_comm_free.argtypes = [C.c_void_p]
    L.mrt_gather_shard_pixels.argtypes = [C.POINTER(MrtRenderDesc), C.POINTER(C.c_uint32)]
    L.mrt_gather_shard_pixels.restype = st
    L.mrt_gather_frame.argtypes = [C.c_void_p, C.POINTER(MrtRenderDesc), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.mrt_gather_frame.restype = st
    L.mrt_render_gather.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(MrtRenderDesc), C.c_void_p, C.POINTER(C.c_uint64)]
    L.mrt_render_gather.restype = st
    _lib = L
    return L


def check(status, what=""):
    if status != 0:
        L = lib()
        raise MrtError(f"{what}: {L.mrt_strerror(status).decode()} ({L.mrt_last_error().decode()})")


# exported symbols declared in include/mrt.h (tests check the library exports every one)
EXPORTS = [
    "mrt_default_params", "mrt_parse_argv", "mrt_select_scene", "mrt_scene_blob_view",
    "mrt_scene_blob_dump_json", "mrt_free_string", "mrt_scene_blob_free", "mrt_init",
    "mrt_scene_upload", "mrt_scene_free", "mrt_default_render_desc", "mrt_local_pixels",
    "mrt_render", "mrt_render_device", "mrt_render_join", "mrt_prepare", "mrt_render_debug", "mrt_progress",
    "mrt_tonemap_argb", "mrt_strerror", "mrt_last_error", "mrt_kernel_ms", "mrt_pack_obj",
    "mrt_scene_kernel_info", "mrt_preview", "mrt_lum_max_device", "mrt_tonemap_device", "mrt_worker_seeds", "mrt_set_worker_seeds",
    "mrt_abi_version", "mrt_comm_unique_id", "mrt_comm_init_rank", "mrt_comm_init_all", "mrt_comm_free",
    "mrt_gather_shard_pixels", "mrt_gather_frame", "mrt_render_gather",
]
