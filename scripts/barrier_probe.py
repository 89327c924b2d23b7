"""Kernel boundary in a replayed graph vs grid barrier in one persistent launch
(scripts/probe/barrier.hip; GPU only): python scripts/barrier_probe.py"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "probe", "libbarrier.so"))
lib.probe_graph_launch.restype = ctypes.c_double
lib.probe_persist.restype = ctypes.c_double
for kind, name in ((0, "empty"), (1, "touch")):
    for grid in (1, 64, 256, 1024):
        print(f"graph launch {name:5s} grid {grid:5d}: {lib.probe_graph_launch(kind, 64, grid, 50):6.2f} us/launch",
              flush=True)
for work in (0, 1):
    for grid in (64, 128, 256, 512):
        print(f"persistent grid {grid:4d} work {work}: {lib.probe_persist(grid, 64, work, 20):6.2f} us/barrier",
              flush=True)
