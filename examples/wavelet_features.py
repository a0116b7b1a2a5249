#!/usr/bin/env python3
"""Wavelet energy features of a batch of signals with the PyTorch ops, and a
gradient through them: a trainable front layer learns to shape the band
energies.  Runs on the GPU when one is visible (HIP kernels), else on the CPU
(the float64 torch definitions of the same ops).

    python examples/wavelet_features.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import models, ops  # noqa: E402


def main():
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    torch.manual_seed(0)
    x = torch.randn(64, 1024, device=dev)

    hi, lo = ops.swt(x, "daubechies", 8, levels=4)          # stationary transform, all levels
    print("swt:", tuple(hi.shape), tuple(lo.shape))
    pyramid = ops.wavedec(x, "symlet", 8, levels=5)          # decimated pyramid in one launch
    print("wavedec:", tuple(pyramid.shape))

    front = torch.nn.Linear(1024, 1024).to(dev)
    feats = models.WaveletEnergyFeatures(levels=4).to(dev)
    target = torch.tensor([4.0, 2.0, 1.0, 0.5, 0.25], device=dev)
    opt = torch.optim.SGD(front.parameters(), lr=0.5)
    for step in range(5):
        e = feats(front(x)).mean(0)                           # band energies, batch mean
        loss = ((e / e.sum() - target / target.sum()) ** 2).sum()
        opt.zero_grad()
        loss.backward()                                       # adjoint filter bank: conv1d kernels
        opt.step()
        print(f"step {step}: loss {loss.item():.6f}")


if __name__ == "__main__":
    main()
