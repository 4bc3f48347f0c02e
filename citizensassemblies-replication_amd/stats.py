"""Consumers of the LEGACY results.

* ``compute_prob_allocation_stats`` / ``upper_confidence_bound``: analysis.py:231-268,
  same arithmetic (the Gini sum in sorted order, scipy's gmean and beta.ppf), host side:
  they read n numbers.
* ``sorted_pair_probabilities``: the curve ``plot_pair_probability_distribution_per_algorithm``
  draws (analysis.py:339-342: ``sorted(histogram.get_dict().values())``, n(n-1)/2 values,
  33.5 M at n = 8192).  For a LEGACY histogram the pair counts are integers <= S, so the
  sorted list is a histogram of the counts: ``pair_histogram_kernel`` bins the upper
  triangle on the device and the host expands ``v / S`` (float64 true division, as the
  reference) ``hist[v]`` times.  Float histograms (LEXIMIN / XMIN portfolios, uniform) are
  sorted on the host.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _native as N


@dataclass
class ProbAllocationStats:
    """analysis.py:61-65."""
    gini: float
    geometric_mean: float
    min: float


def compute_prob_allocation_stats(alloc, cap_for_geometric_mean: bool) -> ProbAllocationStats:
    """analysis.py:231-255 (same summation order, so the same floats)."""
    from scipy.stats import gmean
    n = len(alloc)
    k = round(sum(alloc.values()))
    sorted_probs = sorted(alloc.values())
    gini = sum((2 * i - n + 1) * prob for i, prob in enumerate(sorted_probs)) / (n * k)
    if cap_for_geometric_mean:
        geometric_mean = gmean([max(prob, 1 / 10000) for prob in alloc.values()])
    else:
        geometric_mean = gmean(sorted_probs)
    return ProbAllocationStats(gini=gini, geometric_mean=geometric_mean, min=min(sorted_probs))


def upper_confidence_bound(num_trials: int, sample_proportion: float) -> float:
    """analysis.py:258-268: 99th percentile of the Jeffreys posterior."""
    from scipy.stats import beta
    num_successes = round(sample_proportion * num_trials)
    if num_successes == num_trials:
        return 1.
    return beta.ppf(.99, .5 + num_successes, .5 + num_trials - num_successes)


def pair_count_histogram(d_pairs, n, n_bins, stream=None):
    """hist[v] = number of pairs i < j with count v, from device pair counts (torch int64,
    n*n row-major) via pair_histogram_kernel.  Returns a host uint64 array of n_bins."""
    import torch
    dev = d_pairs.device
    hist = torch.empty(int(n_bins), dtype=torch.int64, device=dev)
    over = torch.empty(1, dtype=torch.int64, device=dev)
    st = stream or torch.cuda.current_stream(dev)
    N.check(N.lib().csa_pair_histogram_async(N.ptr(d_pairs), int(n), N.ptr(hist), int(n_bins), N.ptr(over),
                                             ctypes.c_void_p(st.cuda_stream)))
    st.synchronize()
    if int(over.item()):
        raise ValueError("pair counts exceed n_bins = %d" % n_bins)
    return hist.cpu().numpy().view(np.uint64)


def sorted_counts_to_probabilities(hist, S):
    v = np.flatnonzero(hist)
    return np.repeat(v.astype(np.int64) / S, hist[v].astype(np.int64))


def sorted_pair_probabilities(pair_histogram, device="cuda"):
    """Ascending list of all pair values of a PairHistogram (analysis.py:339-342), as float64."""
    counts, S = getattr(pair_histogram, "_counts", None), getattr(pair_histogram, "_S", None)
    if counts is None or S is None:
        return np.sort(pair_histogram.upper())      # float histogram: not a LEGACY count matrix
    import torch
    n = counts.shape[0]
    if isinstance(counts, np.ndarray):
        d = torch.from_numpy(np.ascontiguousarray(counts, np.int64)).to(device)
    else:
        d = counts.reshape(n, n)              # device counts kept by legacy_probabilities: no host copy
    # every pair count is <= both person counts (the diagonal); the max over the triangle covers
    # matrices whose diagonal was not kept as well
    n_bins = int(torch.triu(d).max().item()) + 1 if n else 1
    return sorted_counts_to_probabilities(pair_count_histogram(d.contiguous().view(-1), n, n_bins), S)
