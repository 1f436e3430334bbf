"""Parsl or a minimal in-process stand-in for it.

The reference declares its aggregation functions as Parsl apps
(`@python_app(executors=["threadpool_executor"])`, decentralized_client.py:383 ...) and its
driver passes AppFutures between them.  When Parsl is installed it is used as is.  When it is
not (this image, the GPU box), this module provides the part of its API the path uses: a
`python_app` decorator whose calls return futures, resolve future arguments before running,
and run on a named thread pool ("threadpool_executor": 2 threads, parsl_setup.py:75-78).
Dependencies are awaited by callbacks, never by blocking a pool thread.
"""
from __future__ import annotations

import threading
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Dict

try:  # pragma: no cover - parsl is absent in this image
    import parsl  # type: ignore
    from parsl.app.app import python_app  # type: ignore

    HAVE_PARSL = True
except Exception:  # noqa: BLE001
    parsl = None
    HAVE_PARSL = False

    _lock = threading.Lock()
    _executors: Dict[str, ThreadPoolExecutor] = {}
    _sizes: Dict[str, int] = {"threadpool_executor": 2, "decentral_train": 1, "experiment": 1}

    def _executor(label: str) -> ThreadPoolExecutor:
        with _lock:
            ex = _executors.get(label)
            if ex is None:
                ex = ThreadPoolExecutor(max_workers=_sizes.get(label, 1), thread_name_prefix=label)
                _executors[label] = ex
            return ex

    def _resolve(x):
        return x.result() if isinstance(x, Future) else x

    def python_app(function=None, executors=("threadpool_executor",), **_ignored):
        label = list(executors)[0] if executors else "threadpool_executor"

        def deco(fn):
            def submit(*args, **kwargs):
                out: Future = Future()

                def run():
                    # a failed dependency's exception surfaces here, through result()
                    try:
                        res = fn(*[_resolve(a) for a in args], **{k: _resolve(v) for k, v in kwargs.items()})
                    except BaseException as exc:  # noqa: BLE001 - propagated into the future
                        out.set_exception(exc)
                    else:
                        out.set_result(res)

                # one callback per distinct dependency still running (a round's apps share most
                # of their futures: ten neighbor futures per aggregation, mostly done already)
                deps = {}
                for a in (*args, *kwargs.values()):
                    if isinstance(a, Future) and not a.done():
                        deps[id(a)] = a
                if not deps:
                    _executor(label).submit(run)
                    return out
                pending = [len(deps)]
                plock = threading.Lock()

                def on_done(_):
                    with plock:
                        pending[0] -= 1
                        ready = pending[0] == 0
                    if ready:
                        _executor(label).submit(run)

                for d in deps.values():
                    d.add_done_callback(on_done)
                return out

            submit.__wrapped__ = fn
            submit.__name__ = getattr(fn, "__name__", "app")
            submit.__doc__ = fn.__doc__
            return submit

        return deco(function) if function is not None else deco

    def configure(sizes: Dict[str, int]) -> None:
        with _lock:
            _sizes.update(sizes)

    def shutdown() -> None:
        with _lock:
            for ex in _executors.values():
                ex.shutdown(wait=True)
            _executors.clear()
