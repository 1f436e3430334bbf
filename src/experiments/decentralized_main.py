"""Single-experiment CLI — mirror of the reference's src/experiments/decentralized_main.py.

Same flags and defaults (reference :25-381); BASELINE config 1 runs it as
    python -m src.experiments.decentralized_main --dataset cifar10 --aggregation_strategy unweighted \
        --rounds 1 --epochs 1 --topology_file <8-ring adjacency>
Executors come from parsl_setup (Parsl when installed, else the in-process stand-in).
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

if __package__ in (None, ""):
    sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

DATASETS = ["mnist", "fmnist", "cifar10", "tiny_mem", "cifar10_augment", "cifar10_augment_vgg", "cifar10_vgg",
            "cifar100_vgg", "cifar10_mobile", "cifar10_vit", "cifar10_resnet18", "cifar10_resnet50",
            "cifar10_dropout", "cifar10_augment_dropout"]
STRATEGY_CHOICES = ["unweighted", "unweighted_fl", "weighted", "test_agg", "scale_agg", "degCent", "betCent",
                    "degCent_sim", "betCent_sim", "random"]

# (flag, type, default, extra argparse kwargs)
_FLAGS = [
    ("--rounds", int, 5, {}), ("--checkpoint_every", int, 3, {}), ("--batch_size", int, 16, {}),
    ("--epochs", int, 2, {}), ("--seed", int, 0, {}), ("--train_test_val", float, None, {"nargs": "+"}),
    ("--lr", float, 1e-3, {}), ("--momentum", float, 0.0, {}), ("--participation", float, 1.0, {}),
    ("--prox_coeff", float, 0, {}), ("--sample_alpha", float, 100, {}), ("--label_alpha", float, 100, {}),
    ("--dataset", str, "mnist", {"choices": DATASETS}),
    ("--tiny_mem_num_labels", int, 50, {"choices": range(1, 101), "metavar": "[1-100]"}),
    ("--aggregation_strategy", str, "unweighted", {"choices": STRATEGY_CHOICES}),
    ("--topology_file", str, "../create_topo/topology/topo_1.txt", {}), ("--out_dir", str, "logs", {}),
    ("--data_dir", str, "../data", {}),
    ("--parsl_executor", str, "experiment_per_node", {"choices": ["polaris_experiment_per_node", "experiment_per_node"]}),
    ("--backdoor_proportion", float, 0.1, {}), ("--backdoor_node_idx", int, 0, {}),
    ("--offset_clients_data_placement", int, 0, {}), ("--centrality_metric_data_placement", str, "degree", {}),
    ("--softmax_coeff", float, 10, {}), ("--gamma", float, 0.95, {}), ("--T_0", float, 66, {}),
    ("--T_mult", float, 1, {}), ("--eta_min", float, 1, {}),
    ("--scheduler", str, None, {"choices": ["exp", "CA", "osc"]}),
    ("--optimizer", str, "sgd", {"choices": ["adam", "sgd", "adamw"]}), ("--weight_decay", float, 0, {}),
    ("--beta_1", float, 0.9, {}), ("--beta_2", float, 0.98, {}), ("--trigger", int, 100, {}),
    ("--num_test", int, 1000, {}), ("--num_example", int, 5000, {}), ("--modulo", int, 16381, {}),
    ("--length", int, 20, {}), ("--max_ctx", int, 150, {}), ("--n_layer", int, 4, {}),
    ("--task_type", str, "multiply", {"choices": ["multiply", "sum"]}),
    ("--data_dis", str, "evens", {"choices": ["evens", "primes"]}),
]
# store_true / store_false switches (reference semantics: --no_train etc. flip a default True)
_SWITCHES = [("--download", "store_false"), ("--no_train", "store_false"), ("--backdoor", "store_true"),
             ("--random_bd", "store_true"), ("--many_to_one", "store_false"),
             ("--non_random_data_placement", "store_false"), ("--softmax", "store_true")]


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    for flag, typ, default, extra in _FLAGS:
        p.add_argument(flag, type=typ, default=default, **extra)
    for flag, action in _SWITCHES:
        p.add_argument(flag, action=action)
    return p


def run_experiment(args) -> int:
    from src.decentralized_app import DecentrallearnApp
    from src.experiments import parsl_setup

    config, _ = parsl_setup.get_parsl_config("local")
    parsl_setup.load(config)
    app = DecentrallearnApp(
        rounds=args.rounds, dataset=args.dataset, batch_size=args.batch_size, epochs=args.epochs, lr=args.lr,
        data_dir=args.data_dir, topology_path=args.topology_file, download=args.download, train=args.no_train,
        label_alpha=args.label_alpha, sample_alpha=args.sample_alpha, participation=args.participation,
        seed=args.seed, log_dir=args.out_dir, aggregation_strategy=args.aggregation_strategy,
        prox_coeff=args.prox_coeff,
        train_test_val=tuple(args.train_test_val) if args.train_test_val is not None else None,
        backdoor=args.backdoor, backdoor_proportion=args.backdoor_proportion,
        backdoor_node_idx=args.backdoor_node_idx, random_bd=args.random_bd, many_to_one=args.many_to_one,
        offset_clients_data_placement=args.offset_clients_data_placement,
        centrality_metric_data_placement=args.centrality_metric_data_placement,
        random_data_placement=args.non_random_data_placement, softmax=args.softmax,
        tiny_mem_num_labels=args.tiny_mem_num_labels, momentum=args.momentum, softmax_coeff=args.softmax_coeff,
        optimizer=args.optimizer, weight_decay=args.weight_decay, beta_1=args.beta_1, beta_2=args.beta_2,
        scheduler=args.scheduler, gamma=args.gamma, T_0=args.T_0, T_mult=args.T_mult, eta_min=args.eta_min,
        trigger=args.trigger, num_test=args.num_test, num_example=args.num_example, modulo=args.modulo,
        length=args.length, max_ctx=args.max_ctx, n_layer=args.n_layer, task_type=args.task_type,
        data_dis=args.data_dis, checkpoint_every=args.checkpoint_every,
    )
    try:
        exit_value = app.run()
    finally:
        parsl_setup.cleanup()
        app.close()
    return exit_value


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    start = time.time()
    rc = run_experiment(args)
    print("Total time: ", time.time() - start)
    return rc


if __name__ == "__main__":
    sys.exit(main())
