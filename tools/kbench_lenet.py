"""Per-kernel timing + ablation of the fused LeNet step (B=128), interleaved rounds in one process.

Each variant is launched N times back-to-back between two events; rounds are interleaved so clock
/ DVFS drift affects all variants alike (cdna_hip_programming.md §5.4 rule 24).  The ``dbg`` masks
are the ablation switches compiled into the kernels (results of skipped parts are kept live).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_example_amd.data import synthetic_mnist  # noqa: E402
from pytorch_distributed_example_amd.engine import LeNetTrainStep  # noqa: E402
from pytorch_distributed_example_amd.models import build_net  # noqa: E402


def main():
    B = int(os.environ.get("KB_B", "128"))
    N = int(os.environ.get("KB_N", "200"))
    R = int(os.environ.get("KB_ROUNDS", "5"))
    dev = torch.device("cuda", 0)
    net = build_net(seed=0, device=dev)
    eng = LeNetTrainStep(net, batch_size=B)
    ds = synthetic_mnist(8192, device=dev)
    eng.bind_dataset(ds.images, ds.labels)
    eng.set_epoch_indices(torch.arange(8192, dtype=torch.int32))
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    K, p, g, e = eng.K, eng.p, eng.g, eng

    def conv_fwd(dbg):
        return lambda: K.lenet_conv_fwd(e.X, e.idx, e.counters[1:], e.nbatches, e.B, e.Y, B, p["conv1.weight"],
                                        p["conv1.bias"], e.Wt2, p["conv2.bias"], e.P1, e.A1, e.P2, e.A2, e.cur_row,
                                        e.cur_lbl, e.bucket_grads[1], dbg)

    def fc_bwd(dbg):
        return lambda: K.lenet_fc_bwd(e.P2, e.H1, e.dZ1, e.dZ2, p["fc1.weight"], B, e.dP2m, g["fc1.weight"],
                                      g["fc1.bias"], g["fc2.weight"], g["fc2.bias"], None, None, None, None,
                                      dbg)

    def conv_bwd(dbg):
        return lambda: K.lenet_conv_bwd(e.X, e.cur_row, e.P1, e.A1, e.dP2m, e.A2, p["conv2.weight"], B,
                                        e.g_c1w_rep, e.g_c1b_rep, g["conv2.weight"], g["conv2.bias"], 16, 576,
                                        e.row_loss, e.row_hit, e.loss_sum, e.correct, dbg)

    variants = {
        "conv_fwd": conv_fwd(0),
        "conv_fwd -conv1": conv_fwd(1),
        "conv_fwd -conv2mfma": conv_fwd(2),
        "conv_fwd -wstage": conv_fwd(4),
        "conv_fwd -all": conv_fwd(7),
        "conv_fwd -chain": conv_fwd(8),
        "conv_fwd -p1store": conv_fwd(16),
        "conv_fwd -zero": conv_fwd(32),
        "conv_fwd -all-chain-p1-zero": conv_fwd(7 | 8 | 16 | 32),
        "fc1_fwd": lambda: K.lenet_fc1_fwd(e.P2, B, p["fc1.weight"], p["fc1.bias"], e.H1, None),
        "head": lambda: K.lenet_head(e.H1, B, p["fc2.weight"], p["fc2.bias"], e.cur_lbl, 1.0 / B, None, e.dZ2, e.dZ1,
                                     e.row_loss, e.row_hit, None, None),
        "fc_bwd": fc_bwd(0),
        "fc_bwd onlyC": fc_bwd(6),
        "fc_bwd onlyA": fc_bwd(5),
        "fc_bwd onlyB": fc_bwd(3),
        "fc_bwd none": fc_bwd(7),
        "conv_bwd": conv_bwd(0),
        "conv_bwd onlyW": conv_bwd(2),
        "conv_bwd onlyD": conv_bwd(1),
        "conv_bwd none": conv_bwd(3),
        "conv_bwd -gatomics": conv_bwd(4),
        "conv_bwd -c1wgrad": conv_bwd(16),
        "conv_bwd -mfma": conv_bwd(32),
        "conv_bwd onlyW -gatom": conv_bwd(2 | 4),
        "conv_bwd onlyW -mfma": conv_bwd(2 | 32),
        "conv_bwd onlyD -mfma-c1": conv_bwd(1 | 16 | 32),
        "conv_bwd onlyD -c1": conv_bwd(1 | 16),
        "adam": lambda: K.adam_flat(e.params, e.grads, e.m, e.v, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, 1.0, e.counters,
                                    e.arrive, -1, e.pack_off, e.Wt2, e.c1_off, 576, 16, 576),
    }
    # whole-step variants: the real producer -> consumer chain (caches / XCD state as in training),
    # with one kernel's roles ablated, to attribute in-step time (isolated launches of the same kernel
    # back-to-back re-read hot inputs and can under-state it by ~2x).
    def step(fc_dbg=0, cv_dbg=0, adam=True, fc_split=False, cf_dbg=0):
        def run():
            conv_fwd(cf_dbg)()
            K.lenet_fc1_fwd(e.P2, B, p["fc1.weight"], p["fc1.bias"], e.H1, None)
            K.lenet_head(e.H1, B, p["fc2.weight"], p["fc2.bias"], e.cur_lbl, 1.0 / B, None, e.dZ2, e.dZ1,
                         e.row_loss, e.row_hit, None, None)
            if fc_split:
                for part in (1, 2):
                    K.lenet_fc_bwd(e.P2, e.H1, e.dZ1, e.dZ2, p["fc1.weight"], B, e.dP2m, g["fc1.weight"],
                                   g["fc1.bias"], g["fc2.weight"], g["fc2.bias"], None, None, None, None,
                                   0, part)
            else:
                fc_bwd(fc_dbg)()
            conv_bwd(cv_dbg)()
            if adam:
                variants["adam"]()
        return run

    variants.update({
        "STEP": step(),
        "STEP fc onlyC": step(fc_dbg=6),
        "STEP fc onlyA": step(fc_dbg=5),
        "STEP fc onlyB": step(fc_dbg=3),
        "STEP fc none": step(fc_dbg=7),
        "STEP fc split C;AB": step(fc_split=True),
        "STEP cv onlyW": step(cv_dbg=2),
        "STEP cv onlyD": step(cv_dbg=1),
        "STEP cv none": step(cv_dbg=3),
        "STEP -adam": step(adam=False),
        "STEP cf -chain": step(cf_dbg=8),
        "STEP cf -p1store": step(cf_dbg=16),
        "STEP cf -zero": step(cf_dbg=32),
        "STEP cf -conv1": step(cf_dbg=1),
        "STEP cf -conv2": step(cf_dbg=2),
    })
    # graph mode: G launches of a variant captured in one hipGraph -> GPU-side cost per launch
    # (kernel + boundary), free of the ~4 us host launch overhead of eager Python launches
    G = int(os.environ.get("KB_G", "20"))
    graphs = {}
    for name, fn in variants.items():
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            fn()
        torch.cuda.current_stream().wait_stream(st)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(G):
                fn()
        graphs[name] = gr
    res = {k: [] for k in variants}
    for r in range(R):
        for name, gr in graphs.items():
            gr.replay()
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(max(1, N // G)):
                gr.replay()
            t.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(t) * 1e3 / (max(1, N // G) * G))
    out = {k: {"median_us": sorted(v)[len(v) // 2], "min_us": min(v)} for k, v in res.items()}
    for k, v in out.items():
        print(f"{k:32s} median {v['median_us']:8.2f} us   min {v['min_us']:8.2f} us")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/kbench_B{B}.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
