"""Per-call drop-in overhead (not part of the product): aggregate_models on pool-bound ResNet-50
models (M = 9, config 3's call) timed against the bare K1 launch, plus a cProfile of the calls.
usage: python tools/percall_profile.py [calls]"""
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    from src.models.resnet import ResNet50
    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd.aggregate import aggregate_models, layout_of_module
    from topology_aware_learning_amd.arena import ModelPool

    dev = torch.device("cuda", 0)
    models = [ResNet50().to(dev) for _ in range(10)]
    pool = ModelPool(layout_of_module(models[0]), 10, dev)
    for i, m in enumerate(models):
        pool.bind(m, i)
    ops_, target = models[:9], models[8]
    w = [1 / 9] * 9
    for _ in range(5):
        aggregate_models(ops_, w, target)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(calls):
        aggregate_models(ops_, w, target)
    torch.cuda.synchronize()
    per_call = (time.perf_counter() - t) / calls * 1e3
    rows = [pool.row_f32(i) for i in range(9)]
    irows = [pool.row_i64(i) for i in range(9)]
    out, out_i = pool.row_f32(8), pool.row_i64(8)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(calls):
        ops.agg_model_f32(rows, irows, w, out, out_i)  # the call's one launch (both segments)
    torch.cuda.synchronize()
    k1 = (time.perf_counter() - t) / calls * 1e3
    print(json.dumps(dict(aggregate_models_ms=round(per_call, 4), bare_k1_ms=round(k1, 4))), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(calls):
        aggregate_models(ops_, w, target)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(20)
    print(s.getvalue())


if __name__ == "__main__":
    main()
