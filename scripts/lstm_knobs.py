#!/usr/bin/env python3
"""Sweep the LSTM hand-off poll back-off knobs (DCA_LSTM_KNOBS) and print per-step fwd/bwd latency."""
import json
import os
import sys

sys.path.insert(0, '.')
from scripts.lstm_latency import bench  # noqa: E402

if __name__ == '__main__':
    cases = [(8, 512), (32, 512), (8, 128)]
    for pre in (0, 12, 24, 40):
        for spin in (0, 2):
            os.environ['DCA_LSTM_KNOBS'] = f'{pre},{spin},{pre},{spin}'
            for B, H in cases:
                r = bench(B, 700, H, reps=3)
                r.update(pre=pre, spin=spin)
                print(json.dumps(r), flush=True)
