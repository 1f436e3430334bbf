"""Checkpointing, future barrier and logging — mirror of the reference's src/utils.py.

The on-disk checkpoint format is the reference's ({"client_state_dicts": [...],
"round_idx": r, "client_results": [...]}, reference utils.py:19-38), so runs are
interchangeable.  State dicts of pool-bound (device-resident) models are copied to host
memory before saving.
"""
from __future__ import annotations

import logging
import pathlib
from concurrent.futures import as_completed
from typing import Optional

import pandas as pd
import torch

from src.aggregation_scheduler import BaseScheduler
from src.decentralized_client import DecentralClient
from src.types import Result
from topology_aware_learning_amd.checkpoint import common_pool, load_state_dicts_into_pool, save_pool_checkpoint

DEFAULT_FORMAT = (
    "%(created)f %(asctime)s %(processName)s-%(process)d "
    "%(threadName)s-%(thread)d %(name)s:%(lineno)d %(funcName)s %(levelname)s: "
    "%(message)s"
)


def save_checkpoint(round_idx: int, clients: list[DecentralClient], client_results: list[Result],
                    ckpt_path: pathlib.Path) -> None:
    """Reference utils.py:19-38.  Models bound to one device ModelPool are written straight
    from the pool (one D2H per segment, topology_aware_learning_amd.checkpoint)."""
    pr = common_pool([c.model for c in clients])
    if pr is not None:
        save_pool_checkpoint(ckpt_path, round_idx, pr[0], pr[1], client_results)
    else:
        sds = [{k: v.detach().to("cpu").clone() for k, v in c.model.state_dict().items()} for c in clients]
        torch.save({"client_state_dicts": sds, "round_idx": round_idx, "client_results": client_results}, ckpt_path)
    print(f"Saved checkpoint for round: {round_idx}")


def load_checkpoint(ckpt_path: pathlib.Path, clients: list[DecentralClient],
                    softmax_coeff_scheduler: BaseScheduler):
    """Restore every client's model and replay the scheduler (reference utils.py:41-56).
    The file is this framework's own (or the reference's) checkpoint; it holds result dicts
    with datetimes, so it is not a weights-only payload."""
    ckpt = torch.load(ckpt_path, map_location=torch.device("cpu"), weights_only=False)
    pr = common_pool([c.model for c in clients])
    if pr is not None:  # pool-bound models: one H2D per segment into their rows
        load_state_dicts_into_pool(pr[0], pr[1], ckpt["client_state_dicts"][: len(clients)])
    else:
        for client, sd in zip(clients, ckpt["client_state_dicts"]):
            client.model.load_state_dict(sd)
    for i in range(ckpt["round_idx"]):
        softmax_coeff_scheduler.step(i)
    return ckpt["round_idx"], clients, ckpt["client_results"], softmax_coeff_scheduler


def process_futures_and_ckpt(client_results: list[Result], train_result_futures, round_states: dict,
                             rounds: int, run_dir: pathlib.Path) -> None:
    """Barrier on all futures, then checkpoint every client's "agg" model as round rounds-1
    and write client_stats.csv (reference utils.py:59-95)."""
    if rounds < (max(round_states.keys()) - 1):
        with open("out.txt", "a") as f:
            print(f"{rounds} < {max(round_states.keys())}", file=f)
        return
    # Clients that were not selected in a round carry a plain (results, client) tuple forward.
    futs = [f for f in train_result_futures if hasattr(f, "result")]
    resolved = [f.result() for f in as_completed(futs)] + [t for t in train_result_futures if isinstance(t, tuple)]
    for r in resolved:
        client_results.extend(r[0])
    ckpt_clients = []
    for _, state in round_states[rounds].items():
        obj = state["agg"]
        ckpt_clients.append(obj[1] if isinstance(obj, tuple) and isinstance(obj[1], DecentralClient) else obj.result()[1])
    save_checkpoint(rounds - 1, ckpt_clients, client_results, f"{run_dir}/{rounds - 1}_ckpt.pth")
    pd.DataFrame(client_results).to_csv(f"{run_dir}/client_stats.csv")


def set_file_logger(filename: str, name: str = "parsl", level: int = logging.DEBUG,
                    format_string: Optional[str] = None) -> logging.Logger:
    logger = logging.getLogger(name)
    logger.setLevel(logging.DEBUG)
    handler = logging.FileHandler(filename)
    handler.setLevel(level)
    handler.setFormatter(logging.Formatter(format_string or DEFAULT_FORMAT, datefmt="%Y-%m-%d %H:%M:%S"))
    logger.addHandler(handler)
    logging.getLogger("concurrent.futures").addHandler(handler)
    return logger
