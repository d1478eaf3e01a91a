"""Synthetic stream generators -- TEST INFRASTRUCTURE ONLY.

Counter-based splitmix64, the same definition as ``generate_kernel`` in
flink_amd/csrc/gwo_kernels.hip, so host-side oracle inputs and device-resident benchmark inputs
are identical record for record:

    u(s, g) = fmix64(seed + s * 0xD1B54A32D192ED03 + (g + 1) * 0x9E3779B97F4A7C15)   (mod 2^64)
    key     = u(0, g) % num_keys                      (key_mode 1: (u(0,g) % (10*num_keys)) % num_keys)
    ts      = t0 + (g // N) * span + ((g % N) * span) // N + u(2, g) % disorder
    value   = u(1, g) % value_range                   (float64: + (u(3, g) >> 11) * 2^-53)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

C1 = np.uint64(0xD1B54A32D192ED03)
C2 = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def fmix(z):
    z = (z ^ (z >> np.uint64(30))) * M1
    z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def u(seed: int, s: int, g: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        return fmix(np.uint64(seed) + np.uint64(s) * C1 + (g.astype(np.uint64) + np.uint64(1)) * C2)


@dataclass
class GenSpec:
    seed: int = 42
    first_index: int = 0
    total_records: int = 1_000_000
    num_keys: int = 10_000
    span_ms: int = 60_000
    disorder_ms: int = 1_000
    t0: int = 0
    value_range: int = 1000
    value_dtype: str = "int64"
    key_mode: int = 0


def generate(spec: GenSpec, n: int, first: int | None = None):
    g = np.arange(n, dtype=np.int64) + (spec.first_index if first is None else first)
    with np.errstate(over="ignore"):
        k0 = u(spec.seed, 0, g)
        if spec.key_mode == 1:
            key = ((k0 % np.uint64(10 * spec.num_keys)) % np.uint64(spec.num_keys)).astype(np.int64)
        else:
            key = (k0 % np.uint64(spec.num_keys)).astype(np.int64)
        jitter = (u(spec.seed, 2, g) % np.uint64(spec.disorder_ms)).astype(np.int64) if spec.disorder_ms > 0 else 0
        q, r = np.divmod(g, spec.total_records)
        ts = spec.t0 + q * spec.span_ms + (r * spec.span_ms) // spec.total_records + jitter
        uv = u(spec.seed, 1, g)
        if spec.value_dtype == "float64":
            val = (uv % np.uint64(spec.value_range)).astype(np.float64) + \
                (u(spec.seed, 3, g) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        else:
            val = (uv % np.uint64(spec.value_range)).astype(np.int64)
    return key, ts.astype(np.int64), val


def punctuated_watermarks(ts: np.ndarray, every: int, lag: int):
    """BoundedOutOfOrdernessWatermarks (CO/api/common/eventtime/BoundedOutOfOrdernessWatermarks.java:57-70):
    after every ``every`` records, ``wm = maxTs - lag - 1``.  Returns (batch end index, wm) pairs."""
    out = []
    running = np.maximum.accumulate(ts) if len(ts) else ts
    for end in range(every, len(ts) + every, every):
        e = min(end, len(ts))
        out.append((e, int(running[e - 1]) - lag - 1))
    return out


def session_stream(num_keys: int, n: int, gap: int = 30_000, lag: int = 5_000, seed: int = 42,
                   late_fraction: float = 0.0, mean_inner: int = 5_000, events_per_session: int = 10,
                   late_extra: int = 0):
    """Config 5: per key, bursts with exponential inner gaps (mean 5 s, capped below
    the session gap) separated by >= gap + 1 ms; arrival order sorted by ts + U[0, lag) (so
    wm = maxTs - lag - 1 never makes an on-time event late); a late variant delays a fraction of
    events by U[lag, 3*lag) (+ late_extra) past that order.  Note a delay below gap + lag is absorbed:
    the late event's own session window [ts, ts + gap) still ends after the watermark.  Returns (key, ts, value, arrival order applied)."""
    rng = np.random.default_rng(seed)
    per = max(1, n // num_keys)
    keys = np.repeat(np.arange(num_keys, dtype=np.int64), per)
    m = len(keys)
    inner = np.minimum(rng.exponential(mean_inner, m), gap - 1).astype(np.int64)
    new_sess = rng.random(m) < 1.0 / events_per_session
    between = (gap + 1 + rng.exponential(gap, m)).astype(np.int64)
    step = np.where(new_sess, between, inner)
    first = np.arange(m) % per == 0
    start = rng.integers(0, 60_000, num_keys)
    step[first] = 0
    ts = np.cumsum(step)
    # restart the cumulative sum at each key
    base = ts[first]
    ts = ts - np.repeat(base, per) + np.repeat(start, per)
    vals = rng.integers(0, 1000, m).astype(np.int64)
    arrival = ts + rng.integers(0, lag, m)
    if late_fraction > 0:
        late = rng.random(m) < late_fraction
        arrival[late] += rng.integers(lag, 3 * lag, int(late.sum())) + late_extra
    order = np.argsort(arrival, kind="stable")
    return keys[order], ts[order], vals[order], arrival[order]


def session_watermarks(arrival_ts: np.ndarray, ts: np.ndarray, every: int, lag: int):
    """Punctuated BoundedOutOfOrderness watermarks over the arrival sequence."""
    return punctuated_watermarks(ts, every, lag)
