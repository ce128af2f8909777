"""Drive scripts/libubench.so on the CSC of the bench's RMAT graph (measurement tool)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd")); sys.path.insert(0, ROOT)
import torch
import pylibcugraph as p
from bench import build_rmat_graph
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libubench.so"))
lib.ubench_gather.restype = ctypes.c_float
lib.ubench_gather.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
h = p.ResourceHandle()
g = build_rmat_graph(p, h, scale)
off, idx, _ = g.adjacency(h, transposed=True)
V, E = off.numel() - 1, idx.numel()
x = torch.rand(V, device="cuda")
rnd = torch.randint(0, V, (E,), device="cuda", dtype=torch.int32)
print(f"V={V} E={E}")
for name, ids in (("csc", idx), ("uniform", rnd)):
    for mode, H in ((0, 0), (1, 0), (2, 0), (3, 8192), (3, 16384), (3, 32768)):
        for blocks in (2048, 8192):
            if mode == 3 and blocks > 2048:
                continue
            ms = lib.ubench_gather(ids.data_ptr(), E, x.data_ptr(), mode, H, blocks, 10)
            print(f"{name:8s} mode {mode} H {H:6d} blocks {blocks:5d}: {ms:.3f} ms  "
                  f"{E/ms/1e6:.1f} Gedge/s  {4*E/ms/1e6:.0f} GB/s idx")
