"""Shared plumbing of the sweep entry-point scripts (torchrun-aware)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.basename(os.path.dirname(os.path.abspath(__file__)))


def package():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    return importlib.import_module(PKG)


def init_distributed():
    """One process per GPU under torchrun; RCCL ("nccl") for the single all-reduce."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist.get_rank()
    return 0


def report(xname, xs, curves, out=None, title="", ylabel="NMSE", logy=True):
    rank = int(os.environ.get("RANK", "0"))
    if rank != 0:
        return
    names = list(curves)
    w = max([14] + [len(n) for n in names])
    print(f"{xname:>8} " + " ".join(f"{n:>{w}}" for n in names))
    for i, x in enumerate(xs):
        print(f"{x:>8} " + " ".join(f"{curves[n][i]:{w}.6e}" for n in names))
    if out:
        import numpy as np
        np.savez(out, x=xs, **{k: v for k, v in curves.items()})
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
            for n in names:
                plt.plot(xs, curves[n], label=n)
            if logy:
                plt.yscale("log")
            plt.xlabel(xname); plt.ylabel(ylabel); plt.title(title)
            plt.grid(True); plt.legend(loc="best")
            plt.savefig(os.path.splitext(out)[0] + ".png")
        except ImportError:
            pass
