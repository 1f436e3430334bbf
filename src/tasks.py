"""Local training / evaluation tasks — minimal mirror of the reference's src/tasks.py.

Training is outside the accelerated path; it exists so the round driver runs end to end.
Deliberate difference: a model bound to the device pool is trained in
place on the GPU and stays there (the reference returns it to the CPU, tasks.py:342, and Parsl
pickles it back), so the following aggregation reads it without any copy.
"""
from __future__ import annotations

import time
from datetime import datetime

import torch
from torch.nn import functional as F
from torch.utils.data import DataLoader

from src._parsl_compat import python_app
from src.types import DataChoices, Result  # noqa: F401
from topology_aware_learning_amd.prox import prox_term


def _device_of(model) -> torch.device:
    for p in model.parameters():
        return p.device
    return torch.device("cpu")


def test_model(model, data, round_idx: int, batch_size: int, seed: int, dataset=None) -> Result:
    device = _device_of(model)
    model.eval()
    loss, correct, n = 0.0, 0, 0
    with torch.no_grad():
        for x, y in DataLoader(data, batch_size=batch_size):
            x, y = x.to(device), torch.as_tensor(y).to(device)
            out = model(x)
            loss += F.cross_entropy(out, y, reduction="sum").item()
            correct += (out.argmax(1) == y).sum().item()
            n += len(y)
    model.train()
    return {"test_loss": loss / max(n, 1), "test_acc": correct / max(n, 1)}


def _train(future, round_idx, epochs, batch_size, lr, momentum, prox_coeff, seed, backdoor, dataset,
           optimizer, weight_decay, beta_1, beta_2, neighbor_futures, with_prox: bool):
    if seed is not None:
        torch.manual_seed(seed)
    client = future[1]
    if getattr(client.model, "_tal_pool", None) is None:
        client.model = client.model.to("cuda" if torch.cuda.is_available() else "cpu")
    device = _device_of(client.model)
    params = list(client.model.parameters())
    if optimizer == "sgd":
        opt = torch.optim.SGD(params, lr=lr, momentum=momentum, weight_decay=weight_decay)
    elif optimizer == "adam":
        opt = torch.optim.Adam(params, lr=lr, weight_decay=weight_decay)
    else:
        opt = torch.optim.AdamW(params, lr=lr, weight_decay=weight_decay, betas=(beta_1, beta_2))
    loader = DataLoader(client.train_data, batch_size=batch_size)
    results = []
    t_epochs = 0.0
    for epoch in range(epochs):
        t0 = time.time()
        client.model.train()
        running = 0.0
        for x, y in loader:
            x, y = x.to(device), torch.as_tensor(y).to(device)
            loss = F.cross_entropy(client.model(x), y)
            running += loss.item()
            if with_prox and prox_coeff > 0:  # FedProx term (reference tasks.py:277-286)
                # pool-bound client + neighbors: one fused pass (topology_aware_learning_amd.prox)
                prox = prox_term(client.model, [nf[1].model for nf in neighbor_futures])
                if prox is None:
                    prox = 0.0
                    for nf in neighbor_futures:
                        for w, wt in zip(client.model.parameters(), nf[1].model.parameters()):
                            prox = prox + (w - wt.to(device)).norm(2)
                loss = loss + (prox_coeff / 2) * prox
            loss.backward()
            opt.step()
            opt.zero_grad()
        t_epochs += time.time() - t0
        res = test_model(client.model, client.global_test_data, round_idx, batch_size, seed, dataset)
        results.append({"avg_time_per_epoch": t_epochs / epochs, "date_time": datetime.now(),
                        "client_idx": client.idx, "neighbors": client.neighbors, "round_idx": round_idx,
                        "epoch": epoch, "data_size": len(client.train_data),
                        "train_loss": running / max(len(loader), 1)} | res)
    if getattr(client.model, "_tal_pool", None) is None:
        client.model.to("cpu")  # reference tasks.py:342 (models not in the device pool)
    return results, client


@python_app(executors=["decentral_train"])
def no_local_train(future, round_idx, epochs, batch_size, lr, momentum, prox_coeff, seed, backdoor=False,
                   dataset=None, optimizer="sgd", weight_decay=5e-4, beta_1=0.9, beta_2=0.98, *neighbor_futures):
    """Reference tasks.py:39-177 (no proximal term)."""
    return _train(future, round_idx, epochs, batch_size, lr, momentum, prox_coeff, seed, backdoor, dataset,
                  optimizer, weight_decay, beta_1, beta_2, neighbor_futures, with_prox=False)


@python_app(executors=["decentral_train"])
def local_train(future, round_idx, epochs, batch_size, lr, momentum, prox_coeff, seed, backdoor=False,
                dataset=None, optimizer="sgd", weight_decay=5e-4, beta_1=0.9, beta_2=0.98, *neighbor_futures):
    """Reference tasks.py:180-343."""
    return _train(future, round_idx, epochs, batch_size, lr, momentum, prox_coeff, seed, backdoor, dataset,
                  optimizer, weight_decay, beta_1, beta_2, neighbor_futures, with_prox=True)
