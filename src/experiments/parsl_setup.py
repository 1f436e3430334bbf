"""Executor configuration — mirror of the reference's src/experiments/parsl_setup.py.

The reference's configs are PBS/Aurora specific (they read $PBS_NODEFILE).  Here:
  * with Parsl installed, get_parsl_config returns a Config with the executor labels the apps
    use: "decentral_train" (training) and "threadpool_executor" (aggregation, 2 threads,
    reference parsl_setup.py:75-78);
  * without Parsl (this image, the GPU box) the in-process stand-in of src._parsl_compat runs
    the same labels and load()/dfk().cleanup() are no-ops.
"""
from __future__ import annotations

import os

from src._parsl_compat import HAVE_PARSL, parsl


def get_parsl_config(parsl_executor: str = "local"):
    node_file = os.getenv("PBS_NODEFILE")
    num_nodes = 1
    if node_file and os.path.exists(node_file):
        with open(node_file) as f:
            num_nodes = len(f.readlines())
    try:
        import torch

        accel = max(1, torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        accel = 1
    if not HAVE_PARSL:
        return None, num_nodes * accel
    from parsl.config import Config  # pragma: no cover - parsl absent in this image
    from parsl.executors import ThreadPoolExecutor

    train = ThreadPoolExecutor(label="decentral_train", max_threads=1)
    agg = ThreadPoolExecutor(label="threadpool_executor", max_threads=2)
    return Config(executors=[train, agg], retries=2), num_nodes * accel


def load(config) -> None:
    if HAVE_PARSL and config is not None:  # pragma: no cover
        parsl.load(config)


def cleanup() -> None:
    if HAVE_PARSL:  # pragma: no cover
        parsl.dfk().cleanup()
    else:
        from src._parsl_compat import shutdown

        shutdown()
