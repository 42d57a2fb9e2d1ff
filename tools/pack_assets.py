#!/usr/bin/env python3
"""Package the reference's scene assets as derived binaries under assets/ (run where
/root/reference exists; the GPU box only receives the repository).

  assets/bunny.mesh, assets/wt_teapot.mesh  parsed OBJ records (mrt_pack_obj: the same parser
                                            select_scene uses; positions are float32 as strtof
                                            yields them), not the OBJ text
  assets/earthmap.rgb.xz                    earthmap.jpg decoded by the reference's own stb_image
                                            v2.28 (oracle/_ref --h-mode texels), xz-compressed;
                                            sha256 of the raw texels is checked on unpack

`python tools/pack_assets.py --unpack` (run by __graft_entry__.build()) restores
assets/earthmap.rgb from the .xz.
"""
import ctypes as C
import hashlib
import lzma
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(ROOT, "assets")
REF = os.environ.get("MRT_REFERENCE", "/root/reference")
EARTH_SHA256 = "b53e1305a076afee4d0e694c20c3a9379ecf192cb79684d64fdeb776b2534464"


def unpack():
    src = os.path.join(ASSETS, "earthmap.rgb.xz")
    dst = os.path.join(ASSETS, "earthmap.rgb")
    if os.path.exists(dst) and os.path.getsize(dst) == 2700 * 1350 * 3:
        return dst
    if not os.path.exists(src):
        return None
    raw = lzma.decompress(open(src, "rb").read())
    if hashlib.sha256(raw).hexdigest() != EARTH_SHA256:
        raise RuntimeError("earthmap texels checksum mismatch")
    with open(dst + ".tmp", "wb") as f:
        f.write(raw)
    os.replace(dst + ".tmp", dst)
    return dst


def pack():
    os.makedirs(ASSETS, exist_ok=True)
    sys.path.insert(0, ROOT)
    from miniraytracer_amd._lib import lib
    L = lib()
    L.mrt_pack_obj.argtypes = [C.c_char_p, C.c_char_p]
    for name in ("bunny", "wt_teapot"):
        st = L.mrt_pack_obj(os.path.join(REF, "obj", name + ".obj").encode(), os.path.join(ASSETS, name + ".mesh").encode())
        assert st == 0, name
    tmp = os.path.join(ASSETS, "earthmap.rgb")
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "mrt_ref_exact"), "--h-mode", "texels", "--h-in",
                    os.path.join(REF, "earthmap.jpg"), "--h-out", tmp], check=True, capture_output=True)
    raw = open(tmp, "rb").read()
    assert hashlib.sha256(raw).hexdigest() == EARTH_SHA256
    with open(os.path.join(ASSETS, "earthmap.rgb.xz"), "wb") as f:
        f.write(lzma.compress(raw, preset=9 | lzma.PRESET_EXTREME))


if __name__ == "__main__":
    if "--unpack" in sys.argv:
        print(unpack())
    else:
        pack()
        print(unpack())
