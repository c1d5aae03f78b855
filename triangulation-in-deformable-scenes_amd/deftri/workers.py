"""Multi-GPU evaluation of the weight search's objective.

deformationOptimization's NLopt Nelder-Mead (g2oBundleAdjustment.cc:491-515) evaluates
outerObjective — an arapOptimization on a Map clone plus calculatePixelsStandDev — one point at a
time.  Every point the next Nelder-Mead step may need (initial simplex; reflection, expansion and
both contractions; shrink points) is known before the step runs (nlopt_nm.nelder_mead(prefetch=)),
so ObjectiveWorkers evaluates such a batch concurrently: one process per GPU (one HIP context and
one deftri context each), replicas of the same device solve on different maps.  Results are
deterministic per point, so the search follows NLopt's sequential path exactly.
"""
import concurrent.futures as cf
import multiprocessing as mp
import pathlib
import sys

_PKG = str(pathlib.Path(__file__).resolve().parent.parent)
_device = None


def _init(devices, counter):
    global _device
    if _PKG not in sys.path:
        sys.path.insert(0, _PKG)
    with counter.get_lock():
        k = counter.value
        counter.value += 1
    _device = devices[k % len(devices)]


def _objective(args):
    x, pmap, settings = args
    from deftri import optimization
    return optimization.outerObjective(x, pmap, settings, device=_device)


class ObjectiveWorkers:
    """`devices`: device ordinal per worker process (e.g. range(torch.cuda.device_count()))."""

    def __init__(self, devices):
        self.devices = list(devices)
        ctx = mp.get_context("spawn")
        self._pool = cf.ProcessPoolExecutor(max_workers=len(self.devices), mp_context=ctx, initializer=_init,
                                            initargs=(self.devices, ctx.Value("i", 0)))

    def map_objective(self, xs, pmap, settings):
        return list(self._pool.map(_objective, [(list(map(float, x)), pmap, settings) for x in xs]))

    def close(self):
        self._pool.shutdown(wait=True)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
