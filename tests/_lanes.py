"""Random and adversarial configurations for the what-if kernels' lane-by-lane oracle checks
(compare >= 256 random lanes per dispatch against the independent Python models,
including overlapping thresholds, min > max, C % P != 0, zero and negative steps, and traces
longer than the 2048-segment LDS staging limit)."""
import numpy as np

S = 1_000_000_000
MS = 1_000_000

ADVERSARIAL = [
    # poll, up_cool, down_cool, up_msgs, down_msgs, up_pods, down_pods, max, min
    (5 * S, 10 * S, 30 * S, 100, 10, 1, 1, 8, 1),            # reference defaults (max 8)
    (5 * S, 12 * S, 7 * S, 100, 150, 1, 1, 8, 1),            # overlapping thresholds, C % P != 0
    (3 * S, 0, 0, 50, 50, 2, 2, 6, 1),                       # equal thresholds, zero cool-downs
    (2 * S, 5 * S, 5 * S, 100, 10, 1, 1, 2, 6),              # min > max
    (4 * S, 9 * S, 11 * S, 100, 10, 0, 0, 8, 1),             # zero steps
    (4 * S, 9 * S, 11 * S, 100, 10, -2, -3, 8, 1),           # negative steps
    (7 * S, 13 * S, 29 * S, -5, -10, 3, 1, 12, 0),           # negative thresholds
    (1 * S, 1 * S, 1 * S, 0, 0, 100, 100, 100, 1),           # main_test.go "ScalingPodNum"
    (6 * S, 600 * S, 45 * S, 300, 5, 1, 4, 16, 2),           # cool-down longer than bursts
    (5 * S, 10 * S, 30 * S, 1 << 40, -(1 << 40), 1, 1, 8, 1),  # thresholds never reached
]


def random_params(m: int, seed: int, min_poll_ms: int = 500) -> np.ndarray:
    """(9, m) int64: the adversarial rows first, then random ones."""
    rng = np.random.default_rng(seed)
    cols = [list(a) for a in ADVERSARIAL]
    while len(cols) < m:
        poll = int(rng.integers(min_poll_ms, 10_000)) * MS
        cool = lambda: int(rng.choice([0, int(rng.integers(0, 120_000)) * MS, poll * int(rng.integers(1, 5))]))
        up = int(rng.integers(-20, 400))
        down = int(rng.integers(-20, 400)) if rng.random() < 0.3 else int(rng.integers(-5, up + 1 if up > -5 else -4))
        mx, mn = int(rng.integers(0, 20)), int(rng.integers(0, 10))
        cols.append([poll, cool(), cool(), up, down, int(rng.integers(-3, 8)), int(rng.integers(-3, 8)), mx, mn])
    return np.ascontiguousarray(np.array(cols[:m], dtype=np.int64).T)


def random_walk_trace(n: int, seed: int, max_step_s: int = 3):
    """n piecewise-constant segments, 1..max_step_s seconds apart, depth a reflected random walk
    crossing the usual thresholds."""
    from kube_sqs_autoscaler_amd.tune import sweep

    rng = np.random.default_rng(seed)
    t = np.concatenate([[0], np.cumsum(rng.integers(1, max_step_s + 1, n - 1)) * S])
    d = np.abs(np.cumsum(rng.integers(-60, 61, n)) + 100) % 600
    return sweep.Trace(t, d)


def lanes_to_check(m: int, k: int, seed: int) -> list:
    """The adversarial lanes plus random others: k in total."""
    rng = np.random.default_rng(seed + 1)
    rest = rng.choice(np.arange(len(ADVERSARIAL), m), size=k - len(ADVERSARIAL), replace=False)
    return list(range(len(ADVERSARIAL))) + sorted(int(i) for i in rest)
