"""Reference-interface mirror of msakarvadia/topology_aware_learning's `src` package.

Same module paths, names and signatures as the reference for the aggregation path
(decentralized_client.py, aggregation_scheduler.py) and the minimal driver around it
(decentralized_app.py, tasks.py, modules.py, utils.py, types.py, experiments/).  The
aggregation arithmetic runs in the MI355X HIP library (topology_aware_learning_amd);
nothing here computes it on the CPU.
"""
