#!/usr/bin/env python3
"""Config 3 (60 s mono STFT) timing as bench.py measures it, for rocprofv3 kernel traces."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

for _ in range(2):
    print(json.dumps(bench.stft_config3()))
