"""Work decomposition of the distributed frame (mirrors what libinsitu_hip.so does on device).

* Volume space: the global volume is cut into bricks (OpenFPM subdomains).  Rank r owns a
  contiguous run of bricks; every brick is one sub-VDI ("virtual rank"), so the set of
  supersegment lists per pixel -- and therefore the image -- does not depend on the number of
  GPUs (DistributedVolumeRenderer.kt:57-63 keeps several grids per compute partner too).
* Image space: P contiguous screen strips along the buffer's slowest axis: x (columns) in VDI
  mode, rank j owning x in [j*W/P, (j+1)*W/P) (VDICompositor.comp:72,
  DistributedVolumes.kt:424-431); rows of the (dim0, dim1) texture in plain mode
  (PlainImageCompositor.comp:70,77, DistributedVolumeRenderer.kt:230-236).
* Exchange: rank s sends strip d of each of its bricks to rank d (one equal-count
  all-to-all); rank d merges V = P*B lists ordered v = s*B + b (virtual rank order, the
  order determineNextSupseg scans, VDICompositor.comp:67).
"""
from __future__ import annotations


def bricks_of_rank(rank: int, nranks: int, n_bricks: int) -> list[int]:
    if n_bricks % nranks:
        raise ValueError(f"{n_bricks} bricks do not split evenly over {nranks} ranks")
    b = n_bricks // nranks
    return list(range(rank * b, (rank + 1) * b))


def strip_of_rank(rank: int, nranks: int, extent: int) -> tuple[int, int]:
    """(offset, width) of rank's screen strip along an axis of `extent` pixels."""
    if extent % nranks:
        raise ValueError(f"{extent} pixels do not split evenly into {nranks} strips")
    w = extent // nranks
    return rank * w, w


def list_order(nranks: int, bricks_per_rank: int) -> list[tuple[int, int]]:
    """(source rank, local brick slot) of merged list v = s*B + b."""
    return [(s, b) for s in range(nranks) for b in range(bricks_per_rank)]
