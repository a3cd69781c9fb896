#!/usr/bin/env python3
"""One line per bench.py JSON log: frames/s, ms per frame, render stage split, latency, pipeline depth.
usage: tools/bench_lines.py gpurun_out/<name>.log ..."""
import json
import sys

for path in sys.argv[1:]:
    try:
        lines = [ln for ln in open(path) if ln.startswith("{")]
    except OSError as e:
        print(f"{path}: {e}")
        continue
    for ln in lines:
        d = json.loads(ln)
        c, st = d["config"], d["config"]["stage_ms"]
        print(f"{path.split('/')[-1]:24s} {d['value']:8.2f} fps {d['ms_per_step']:7.3f} ms  render {st['render']:7.3f} "
              f"(sample {st['render.sample_kernel']:6.3f} search {st['render.search_kernel']:6.3f})  "
              f"composite {st['composite']:6.3f}  depth {c.get('pipeline_depth')}  latency {c.get('frame_latency_ms')} "
              f"host {c.get('frame_latency_host_ms')}  frac {d['roofline']['frac']:.3f}")
