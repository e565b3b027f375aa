#!/usr/bin/env python3
"""Diagnostic: keep the GPU busy with a stream of tiny kernels for S seconds
(light load on every CU), so that a lone launch in another process can be
timed with the device out of its idle clock state.  usage: heater.py S"""
import sys
import time

import torch

s = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
x = torch.zeros(1 << 16, device="cuda")
t_end = time.time() + s
while time.time() < t_end:
    for _ in range(200):
        x.add_(1.0)
    torch.cuda.synchronize()
