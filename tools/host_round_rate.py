"""Host-memory path, one round (not part of the product): 64 CPU ResNet-50 models (the
reference's placement after training), random 8-regular graph, 64 per-call aggregations in
client order, without and with the opt-in operand cache (TAL_HOST_CACHE_GB), then with the models
bound to pinned host rows (TAL_HOST_PIN; bound on the warm-up call, the steady state is timed).
usage: python tools/host_round_rate.py [rounds]"""
import json
import os
import sys
import time
from pathlib import Path

import networkx as nx
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from src.models.resnet import ResNet50
    from topology_aware_learning_amd import aggregate

    torch.manual_seed(0)
    models = [ResNet50() for _ in range(64)]
    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    n = sum(v.numel() for v in models[0].state_dict().values())
    for pin, gb in (("0", "0"), ("0", "16"), ("1", "0"), ("1", "16")):
        os.environ["TAL_HOST_CACHE_GB"] = gb
        os.environ["TAL_HOST_PIN"] = pin
        aggregate.aggregate_models([models[j] for j in orders[0]], [1 / 9] * 9, models[0])  # warm
        if pin == "1":  # bind every model (one host copy each) before timing
            for i, o in enumerate(orders):
                aggregate.aggregate_models([models[j] for j in o], [1 / len(o)] * len(o), models[i])
        ts = []
        for _ in range(rounds):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i, o in enumerate(orders):
                aggregate.aggregate_models([models[j] for j in o], [1 / len(o)] * len(o), models[i])
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        c = aggregate._host_cache()
        print(json.dumps(dict(host_pin=pin == "1", host_cache_gb=float(gb), ms_per_round=[round(1e3 * x, 1) for x in ts],
                              ms_per_call=round(1e3 * min(ts) / 64, 2),
                              params_per_s=64 * n / min(ts),
                              hits=c.hits if c else None, misses=c.misses if c else None)), flush=True)


if __name__ == "__main__":
    main()
