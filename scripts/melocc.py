#!/usr/bin/env python3
"""Workgroups per CU of the fused mel kernels (k_stft_pair MODE 3 / 4) against
their dynamic LDS bytes (scripts/stftlab.hip lab_mel_occupancy)."""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch.zeros(1, device="cuda")
lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
lib.lab_mel_occupancy.argtypes = [ctypes.c_int, ctypes.c_longlong]
for mode in (3, 4):
    print(mode, [(d, lib.lab_mel_occupancy(mode, d)) for d in (0, 4208, 5120, 6084, 6336, 6340, 6400, 7168, 7701, 8192)])
