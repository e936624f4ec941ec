"""Driver of scripts/studies/packet_sim.cpp (round-6 study: coherent primary-ray packets).

usage: python scripts/studies/packet_run.py c3 [ntiles] [frames]
Writes the scene to /tmp/packet_scene.bin, runs /tmp/packet_sim (build line in packet_sim.cpp) and prints its counts
plus the lane-slot model of the kernel cost.
"""
import json
import struct
import subprocess
import sys

sys.path[:0] = ['/root/repo', '/root/repo/hello-raytracing_amd', '/root/repo/tests']
import numpy as np  # noqa: E402
import scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
ntiles = sys.argv[2] if len(sys.argv) > 2 else "400"
frames = sys.argv[3] if len(sys.argv) > 3 else "4"
sd = scenes.CONFIGS[cfg]()
cam = np.ascontiguousarray(sd.camera).tobytes()
sph = np.ascontiguousarray(sd.spheres).tobytes()
assert len(cam) == 80 and len(sph) % 48 == 0
with open("/tmp/packet_scene.bin", "wb") as f:
    f.write(cam + struct.pack("<I", len(sph) // 48) + sph)
    if sd.bvh is not None:  # the triangle / mixed program: (sizes, nodes, triangles, materials)
        nodes, tris, mats = (np.ascontiguousarray(x) for x in sd.bvh[1:])
        f.write(struct.pack("<4I", sd.mode, len(nodes), len(tris), len(mats)) + nodes.tobytes() + tris.tobytes()
                + mats.tobytes())
out = subprocess.run(["/tmp/packet_sim", "/tmp/packet_scene.bin", str(sd.width), str(sd.height), str(sd.bounces or 50),
                      ntiles, frames], capture_output=True, text=True, check=True).stdout
print(out, end="")
if "HJSON" in out:
    h = json.loads(out.split("HJSON ", 1)[1].split("\n", 1)[0])
    print(f"heap walk: primary per-lane steps {h['hp']:.1f}, union {h['hu']:.1f} per packet of {h['rpp']:.0f} "
          f"({h['hu'] / h['hp']:.2f}x one walk; {h['hul']:.1f} lanes per union step)")
if "\nJSON" not in out:
    sys.exit(0)
j = json.loads(out.split("\nJSON ", 1)[1])
# lane-slot model (diag counters of k_trace_split at suspend_below 24, profiles/r05/diag_c/diag_split_c3.log):
# a per-lane box step costs 1 / 0.607 lane slots, a leaf step 1 / 0.586; a packet step costs 64 lane slots for the
# rays_per_packet queries it serves (every lane runs it)
UB, UL = 0.607, 0.586
fp = j["qp"] / j["q"]
now_p = j["pbox"] / UB + j["pleaf"] / UL
pk_p = (j["ubox"] * 64 + j["uleaf"] * 64) / j["rays_per_packet"] / 64 * 64 / 64
pk_p = (j["ubox"] + j["uleaf"]) * 64 / j["rays_per_packet"]
now_s = j["sbox"] / UB + j["sleaf"] / UL
walk_now = fp * now_p + (1 - fp) * now_s
walk_pk = fp * pk_p + (1 - fp) * now_s
print(f"lane slots per primary query: today {now_p:.2f}, packet {pk_p:.2f} (steps x 64 / rays per packet)")
print(f"walk lane slots per query: today {walk_now:.2f}, packet {walk_pk:.2f}: walk {100 * (walk_pk / walk_now - 1):+.1f} %")
# leaf steps cost more than box steps: weight a leaf step by its sphere tests (~25 VALU each vs ~50 per box step)
sph_pk = j["usph"] * 64 / j["rays_per_packet"]
print(f"sphere tests per primary query: today {j['psph']:.2f} (lane, at leaf util {UL}: {j['psph'] / UL:.2f} slots), "
      f"packet {sph_pk:.2f} slots")
