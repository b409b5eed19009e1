"""Capture one btb training step as run_epoch does (graphs.py) and dump the
captured hipGraph's nodes and dependency edges, WITHOUT replaying it.

VERDICT r3 item 7: before 6e755f9 the library issued hipMemsetAsync /
hipMemcpyAsync inside the captured step, and replays gave wrong edge-weight
gradients (once a garbage pair index and a fault).  Run with

    GGNN_LIB=tools/libggnn_memset.so python tools/capture_probe.py

where tools/libggnn_memset.so (tools/build_memset_probe_lib.py) is libggnn
with fill_async / copy_async as hipMemsetAsync / hipMemcpyAsync, the
round-2 form, to see whether every memset / memcpy node
is ordered after its producer and before its consumer; without GGNN_LIB it
dumps the shipped kernel-only graph.  The step: the reference's default
model at hidden 400 (general path, pair mode), T = 4, the training feed's
dropouts, edge-list batches of the reference's own dev sentences.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
         7: "event_record", 10: "mem_alloc", 11: "mem_free"}


class Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class KernelNodeParams(ctypes.Structure):
    _fields_ = [("blockDim", Dim3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p), ("gridDim", Dim3),
                ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]


class MemsetParams(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


def walk(graph_handle):
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipKernelNameRefByPtr.restype = ctypes.c_char_p
    g = ctypes.c_void_p(graph_handle)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) == 0
    index = {nodes[i]: i for i in range(n.value)}
    table = []
    for i in range(n.value):
        t = ctypes.c_int(0)
        assert hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)) == 0
        nd = ctypes.c_size_t(0)
        assert hip.hipGraphNodeGetDependencies(ctypes.c_void_p(nodes[i]), None, ctypes.byref(nd)) == 0
        deps = []
        if nd.value:
            arr = (ctypes.c_void_p * nd.value)()
            assert hip.hipGraphNodeGetDependencies(ctypes.c_void_p(nodes[i]), arr, ctypes.byref(nd)) == 0
            deps = sorted(index[arr[j]] for j in range(nd.value))
        e = {"i": i, "type": TYPES.get(t.value, str(t.value)), "deps": deps}
        if t.value == 0:
            kp = KernelNodeParams()
            if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(nodes[i]), ctypes.byref(kp)) == 0:
                nm = hip.hipKernelNameRefByPtr(ctypes.c_void_p(kp.func), None)
                e["name"] = (nm.decode() if nm else hex(kp.func or 0))[:60]
                e["grid"] = [kp.gridDim.x, kp.gridDim.y, kp.gridDim.z]
        elif t.value == 2:
            mp = MemsetParams()
            assert hip.hipGraphMemsetNodeGetParams(ctypes.c_void_p(nodes[i]), ctypes.byref(mp)) == 0
            e.update(dst=hex(mp.dst or 0), elementSize=mp.elementSize, width=mp.width, height=mp.height,
                     value=hex(mp.value))
        table.append(e)
    return table


def main():
    import torch
    from ggnn_amd.model import DenseGGNNChemModel

    keep_graph = torch.cuda.CUDAGraph

    class KeptGraph(keep_graph):
        def __new__(cls, *a, **k):
            return keep_graph.__new__(cls, keep_graph=True)

        def __init__(self, *a, **k):
            super().__init__(keep_graph=True)

        def replay(self):          # capture only: never launched
            KeptGraph.replays_skipped += 1

    KeptGraph.replays_skipped = 0
    torch.cuda.CUDAGraph = KeptGraph

    g = np.load(os.path.join(ROOT, "tests", "golden", "batching_golden.npz"))
    data = json.loads(str(g["raw_json"]))
    vocab = 1 + max(max(d["words_index"]) for d in data)
    m = DenseGGNNChemModel(params={"hidden_size": 400, "num_timesteps": 4, "batch_size": 8,
                                   "compact_adjacency": True, "edge_weight_dropout_keep_prob": 0.9},
                           num_edge_types=int(g["num_edge_types"]), output_size_edges=int(g["output_size_edges"]),
                           pos_size=int(g["pos_size"]), bucket_max_nodes=int(g["bucket_max_nodes"]),
                           precision="fp32", vocab_size=vocab)
    feed = next(iter(m.make_minibatch_iterator(m.process_raw_graphs(data, True), True)))
    feed["out_layer_dropout_keep_prob"] = m.params["out_layer_dropout_keep_prob"]
    m.train_step(dict(feed))            # the shape's first batch: its body, eagerly
    m.train_step(dict(feed))            # second: captured (replay skipped)
    torch.cuda.synchronize()
    cs = next(iter(m._graphs.values()))
    table = walk(cs.graph.raw_cuda_graph())
    lib = os.environ.get("GGNN_LIB", "ggnn_amd/libggnn.so")
    print("library:", lib, " replays skipped:", KeptGraph.replays_skipped, " nodes:", len(table))
    for e in table:
        extra = ""
        if e["type"] == "kernel":
            extra = "%s grid %s" % (e.get("name"), e.get("grid"))
        elif e["type"] == "memset":
            extra = "dst %s width %d x elementSize %d value %s" % (e["dst"], e["width"], e["elementSize"], e["value"])
        print("%4d %-12s deps %-12s %s" % (e["i"], e["type"], e["deps"], extra))
    # the checks: a single chain (every node depends on exactly the node
    # captured before it), and each memset / memcpy node between its neighbours
    dependents = {e["i"]: [] for e in table}
    for e in table:
        for d in e["deps"]:
            dependents[d].append(e["i"])
    chain = all(e["deps"] == ([e["i"] - 1] if e["i"] else []) for e in table)
    odd = [e for e in table if e["type"] in ("memset", "memcpy")
           and (e["deps"] != [e["i"] - 1] or dependents[e["i"]] != [e["i"] + 1])]
    print("types:", {t: sum(1 for e in table if e["type"] == t) for t in set(e["type"] for e in table)})
    print("single chain in capture order:", chain)
    print("memset/memcpy nodes not between their capture-order neighbours:", [e["i"] for e in odd])


if __name__ == "__main__":
    main()
