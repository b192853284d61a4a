#!/usr/bin/env python3
"""Does torch.cuda.synchronize() (hipDeviceSynchronize) wait for the engine's own non-blocking HIP streams?
Runs 2000 generations at 32768^2 (~20 ms of GPU work), calls torch.cuda.synchronize() only, and then
checks with the engine's progress query that no GPU work is outstanding (and that the host waited as
long as the work takes)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gol_amd  # noqa: E402

torch.cuda.synchronize()
sim = gol_amd.Simulation(32768, backend="hip", device=0).init(pattern=5, seed=1)
sim.step(8)
sim.synchronize()
t0 = time.perf_counter()
sim.step(2000)
t_enq = time.perf_counter() - t0
torch.cuda.synchronize()
t_sync = time.perf_counter() - t0
idle = sim.engine.gpu_idle()
print(f"sync_check: enqueue {t_enq * 1e3:.2f} ms, torch sync returned after {t_sync * 1e3:.2f} ms, engine streams idle: {idle}")
sys.exit(0 if idle else 1)
