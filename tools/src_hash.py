#!/usr/bin/env python3
"""Hash of the sources a profile's kernels are built from (scenery-insitu_amd/csrc/*, its Makefile and
include/insitu_hip.h): tools/prof_summary.py stores it in summary.json["_config"]["csrc_sha16"], bench.py
compares it with the tree it runs from before it quotes the profile's traffic and VALU figures."""
from __future__ import annotations

import hashlib
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def csrc_hash(root: Path = ROOT) -> str:
    files = sorted((root / "scenery-insitu_amd" / "csrc").glob("*")) + \
        [root / "scenery-insitu_amd" / "Makefile", root / "include" / "insitu_hip.h"]
    h = hashlib.sha256()
    for f in files:
        if f.is_file():
            h.update(f.relative_to(root).as_posix().encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(csrc_hash())
