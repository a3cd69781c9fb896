#!/usr/bin/env python3
"""Instruction counts per kernel of a gfx950 assembly file (hipcc --cuda-device-only -S): LDS, VMEM,
VALU/SALU totals, and the register/spill metadata -- a static check of a layout or loop change before
it goes to the GPU.  usage: tools/asm_stats.py file.s [name-substring ...]"""
import re
import sys

KINDS = ["ds_read_b32", "ds_read2_b32", "ds_read_b64", "ds_read2_b64", "ds_read_b128", "ds_write",
         "global_load_dword ", "global_load_dwordx2", "global_load_dwordx4", "global_store", "buffer_load",
         "s_waitcnt", "v_", "s_"]


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    text = open(path).read()
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n((?:\s+\.[\w_]+:.*\n)+)", text):
        d = dict(re.findall(r"\.([\w_]+):\s+(\S+)", m.group(2)))
        meta[m.group(1)] = d
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end", text, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if subs and not any(s in name for s in subs):
            continue
        lines = [ln.strip() for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", "."))]
        cnt = {k: sum(1 for ln in lines if ln.startswith(k)) for k in KINDS}
        md = meta.get(name, {})
        print(f"{name[:70]}  vgpr {md.get('vgpr_count', '?')} spill {md.get('vgpr_spill_count', '?')} "
              f"lines {len(lines)}")
        print("   " + "  ".join(f"{k.strip()}={v}" for k, v in cnt.items() if v))


if __name__ == "__main__":
    main()
