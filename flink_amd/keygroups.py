"""Key-group partitioning: ``KeyGroupRange`` + the GPU-side ``KeyGroupRangeAssignment``.

Host-side range arithmetic follows flink-runtime/src/main/java/org/apache/flink/runtime/state/
KeyGroupRangeAssignment.java:88-137 and KeyGroupRange.java:54-99; per-key assignment runs in the
gfx950 key-group kernel (bit-exact murmurHash, ``gwo_assign_key_groups``).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N

UPPER_BOUND_MAX_PARALLELISM = 1 << 15   # CO/api/dag/Transformation.java:99
DEFAULT_LOWER_BOUND_MAX_PARALLELISM = 1 << 7


@dataclass(frozen=True)
class KeyGroupRange:
    start_key_group: int
    end_key_group: int

    def contains(self, kg: int) -> bool:
        return self.start_key_group <= kg <= self.end_key_group

    def number_of_key_groups(self) -> int:
        return max(0, self.end_key_group - self.start_key_group + 1)


def _round_up_pow2(x: int) -> int:
    p = 1
    while p < x:
        p <<= 1
    return p


def compute_default_max_parallelism(parallelism: int) -> int:
    """KeyGroupRangeAssignment.java:129-137."""
    if parallelism <= 0 or parallelism > UPPER_BOUND_MAX_PARALLELISM:
        raise ValueError("Operator parallelism not within bounds")
    return min(max(_round_up_pow2(parallelism + parallelism // 2), DEFAULT_LOWER_BOUND_MAX_PARALLELISM),
               UPPER_BOUND_MAX_PARALLELISM)


def compute_key_group_range_for_operator_index(max_parallelism: int, parallelism: int, index: int) -> KeyGroupRange:
    """KeyGroupRangeAssignment.java:88-101."""
    if not (0 < parallelism <= UPPER_BOUND_MAX_PARALLELISM and 0 < max_parallelism <= UPPER_BOUND_MAX_PARALLELISM):
        raise ValueError("parallelism out of bounds")
    if max_parallelism < parallelism:
        raise ValueError("Maximum parallelism must not be smaller than parallelism.")
    start = (index * max_parallelism + parallelism - 1) // parallelism
    end = ((index + 1) * max_parallelism - 1) // parallelism
    return KeyGroupRange(start, end)


def assign_key_groups(keys, max_parallelism: int, parallelism: int = 1, key_kind: str = "long", device: int = 0):
    """GPU kernel: key groups and operator indices of an int64 key column (numpy in/out)."""
    k = np.ascontiguousarray(keys, dtype=np.int64)
    kg = np.empty(len(k), np.int32)
    op = np.empty(len(k), np.int32)
    st = N.lib().gwo_assign_key_groups(k.ctypes.data_as(C.c_void_p), len(k),
                                       N.KEY_INT if key_kind == "int" else N.KEY_LONG, max_parallelism,
                                       parallelism, kg.ctypes.data_as(C.c_void_p), op.ctypes.data_as(C.c_void_p),
                                       device)
    N.check(st, None, "gwo_assign_key_groups")
    return kg, op


def encode_utf16(keys):
    """Strings -> (UTF-16 code units, int64 offsets): the columnar form a host hands over (a Java String's
    chars; lone surrogates pass through as code units, as in Java)."""
    enc = [k.encode("utf-16-le", "surrogatepass") for k in keys]
    offsets = np.zeros(len(enc) + 1, np.int64)
    if enc:
        offsets[1:] = np.cumsum([len(b) // 2 for b in enc])
    chars = np.frombuffer(b"".join(enc), dtype=np.uint16).copy() if offsets[-1] else np.zeros(1, np.uint16)
    return chars, offsets


def decode_utf16(chars, offsets):
    b = np.ascontiguousarray(chars, np.uint16).tobytes()
    return [b[2 * offsets[i]:2 * offsets[i + 1]].decode("utf-16-le", "surrogatepass") for i in range(len(offsets) - 1)]


def assign_key_groups_strings(keys, max_parallelism: int, parallelism: int = 1, device: int = 0):
    """GPU kernel: String.hashCode (UTF-16 code units), key groups and operator indices of String keys.
    The strings are packed as one UTF-16 code-unit array plus int64 offsets (the columnar form a host
    would hand over)."""
    chars, offsets = encode_utf16(keys)
    n = len(offsets) - 1
    h = np.empty(n, np.int32)
    kg = np.empty(n, np.int32)
    op = np.empty(n, np.int32)
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    st = N.lib().gwo_assign_key_groups_utf16(P(chars), P(offsets), n, max_parallelism, parallelism, P(h),
                                             P(kg), P(op), device)
    N.check(st, None, "gwo_assign_key_groups_utf16")
    return h, kg, op


def window_starts(ts, offset: int, size: int, device: int = 0):
    """GPU kernel: ``TimeWindow.getWindowStartWithOffset`` over a timestamp column."""
    t = np.ascontiguousarray(ts, dtype=np.int64)
    out = np.empty(len(t), np.int64)
    st = N.lib().gwo_window_starts(t.ctypes.data_as(C.c_void_p), len(t), offset, size,
                                   out.ctypes.data_as(C.c_void_p), device)
    N.check(st, None, "gwo_window_starts")
    return out
