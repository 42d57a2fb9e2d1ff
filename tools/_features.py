import sys
sys.path.insert(0, ".")
import miniraytracer_amd as m
names = ["BVH", "MESH", "VOLUME", "INST", "TEX", "METAL", "ISO", "MOVING", "SKY", "BSPHERE", "UV", "LIN", "BVHW"]
for sid in range(10):
    r = m.Renderer(m.select_scene(sid, 1.0), 0)
    ki = r.kernel_info()
    f = ki["features"]
    print(sid, [n for i, n in enumerate(names) if f >> i & 1], "sig", f >> 16, "kernel", hex(ki["kernel_features"]), "vgprs", ki["vgprs"], "grid", ki["grid"], "lds", ki["lds_bytes"])
