"""Convergence records on disk: the file surface the reference's ``compare.py`` reads.

compare.py:7-10 loads four 1-D float text files from ``settings.Dir_PERFORMANCE``
(``$HOME/Documents/convex_optimization/Performance``, settings.py:19):
``GPU_time.txt``, ``GPU_errors.txt``, ``CPU_time.txt``, ``CPU_errors.txt``, then
plots log10(error) against time (compare.py:12-21).  Nothing in the reference
writes them; ``save_performance`` does, from a driver's ``time_iter`` /
``err_iter`` arrays (lasso.py:54-62), and ``compare_figure`` draws compare.py's
figure into a file.  (average.py, which averages records over instances, is out of
scope: SURVEY.md section 2.)
"""
import os

import numpy as np


def default_dir():
    return os.path.join(os.path.expanduser("~"), "Documents", "convex_optimization", "Performance")


def trim_records(time_iter, err_iter, iters=None):
    """Cut the ITER_MAX(+1)-long record arrays to the iterations actually run.

    ``time_iter[t + 1]`` is the time after iteration t and ``err_iter[t]`` its
    error (lasso.py:54-62), so the pair (time_iter[1:n+1], err_iter[:n]) is
    what compare.py plots.
    """
    t = np.asarray(time_iter, dtype=np.float64).reshape(-1)
    e = np.asarray(err_iter, dtype=np.float64).reshape(-1)
    n = len(e) if iters is None else int(iters)
    return t[1:n + 1], e[:n]


def save_performance(prefix, time_iter, err_iter, directory=None, iters=None):
    """Write <prefix>_time.txt and <prefix>_errors.txt (prefix 'GPU' or 'CPU')."""
    d = directory or default_dir()
    os.makedirs(d, exist_ok=True)
    t, e = trim_records(time_iter, err_iter, iters)
    np.savetxt(os.path.join(d, f"{prefix}_time.txt"), t)
    np.savetxt(os.path.join(d, f"{prefix}_errors.txt"), e)
    return os.path.join(d, f"{prefix}_time.txt"), os.path.join(d, f"{prefix}_errors.txt")


def load_performance(directory=None):
    """The four arrays compare.py loads (compare.py:7-10); missing files are skipped."""
    d = directory or default_dir()
    out = {}
    for dev in ("GPU", "CPU"):
        for kind in ("time", "errors"):
            path = os.path.join(d, f"{dev}_{kind}.txt")
            if os.path.exists(path):
                out[f"{dev.lower()}_{kind}"] = np.atleast_1d(np.loadtxt(path))
    return out


def compare_figure(directory=None, out_path=None):
    """compare.py:12-21: log10(error) vs time, CPU blue / GPU red, saved to ``out_path``."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    data = load_performance(directory)
    fig, ax = plt.subplots()
    for dev, color in (("cpu", "blue"), ("gpu", "red")):
        if f"{dev}_time" in data and f"{dev}_errors" in data:
            ax.plot(data[f"{dev}_time"], np.log10(data[f"{dev}_errors"]), label=dev.upper(), color=color)
    ax.legend(loc="upper right", fontsize="x-large")
    ax.set_xlabel("time/s")
    ax.set_ylabel("errors/log10")
    out_path = out_path or os.path.join(directory or default_dir(), "compare.png")
    fig.savefig(out_path)
    plt.close(fig)
    return out_path

