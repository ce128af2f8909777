import sys, os
sys.path.insert(0, "cugraph-forked_amd"); sys.path.insert(0, ".")
if sys.argv[1] == "torch_first":
    import torch
import numpy as np
import pylibcugraph as plc
import torch
h = plc.ResourceHandle()
g = plc.SGGraph(h, plc.GraphProperties(), np.array([0,1,2],np.int32), np.array([1,2,0],np.int32), None, store_transposed=True)
print(plc.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 100, False)[1])
import re
maps = open("/proc/self/maps").read()
print(sorted(set(re.findall(r"\S*(?:amdhip64|hsa-runtime64|rccl)\S*", maps))))
