import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_cuda_process_amd as m
prob = m.heat3d(nx=64, ny=16, nz=20)
for ranks in (1, 3):
    print("ranks", ranks, flush=True)
    with m.Simulation(prob, device="hip", ranks=ranks, graph=True) as sim:
        sim.init(); sim.run(6); sim.synchronize()
        print("ok", float(sim.gather().sum()), flush=True)
