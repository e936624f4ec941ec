"""Driver of scripts/studies/heap_cull_sim.c (round-5 study of culling the reference heap walk)."""
import sys, time, ctypes as C
sys.path[:0] = ['/root/repo', '/root/repo/hello-raytracing_amd', '/root/repo/tests']
import scenes
from oracle import oracle as O
L = C.CDLL('/tmp/liboracle_cull.so')  # built from scripts/studies/heap_cull_sim.c (header)
L.oracle_render.restype = C.c_uint64
L.oracle_render.argtypes = [C.POINTER(O.OParams), C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_uint64)]
L.cull_stat.restype = C.c_uint64
L.cull_config.argtypes = [C.c_int, C.c_float, C.c_float, C.c_int]
O._libs[99] = L
cfg = sys.argv[1]
batch, mrel, mabs, limit = int(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5])
L.cull_config(batch, mrel, mabs, limit)
sd = scenes.CONFIGS[cfg]()
t = time.time()
_, q = scenes.oracle_render(sd, rows=(4, sd.height // 24, 24), frames=4, threads=8, contract=99)
st = [L.cull_stat(i) for i in range(10)]
walks = st[9]
print(f"{cfg} batch {batch} margin {mrel}/{mabs} limit {limit}: walks {walks}, ref steps/walk {st[0]/walks:.2f} (nodes {st[1]/walks:.2f}, tris {st[2]/walks:.2f}); culled steps/walk {st[4]/walks:.2f}, tris {st[5]/walks:.2f}; fallbacks {st[3]} ({st[3]/walks:.2e}); mismatches {st[6]}; {time.time()-t:.1f}s")
