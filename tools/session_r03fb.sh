#!/bin/bash
# Round 3: fast pass restart, second try (children reset on the batched restart too)
tools/gpu_session.sh \
 "ab|400|tools/variant_ab.sh fr0" \
 "emu|300|tools/emu_ab.sh fr0" \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
