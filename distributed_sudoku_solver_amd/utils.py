"""Host-side mirror of utils.py:1-9 (the reference's work-partition rule).

find_next_empty / is_valid (utils.py:14-56) have no host counterpart: the HIP
solver evaluates them (as bitmask propagation) on the device.
"""


def split_array_in_middle(arr):
    """(arr[:len//2], arr[len//2:]) -- utils.py:1-9.  On a `range` this yields two
    contiguous digit ranges, i.e. two disjoint first-cell masks (engine.range_to_mask)."""
    h = len(arr) // 2
    return arr[:h], arr[h:]
