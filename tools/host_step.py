"""Is a batched bench config host-bound? Host enqueue time of K timed steps (perf_counter around the launch loop,
no synchronisation inside it) next to their device time (until torch.cuda.synchronize() returns).

    python tools/host_step.py C2 C3 [--steps 60]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    cfgs = [c for c in sys.argv[1:] if not c.startswith("--")]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 60
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda:0")
    for cfg in cfgs:
        W = bench.setup_workload(cfg, a, dev, 0, False)
        bench.warm_workload(W, a)
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                bench._step(W, i, False)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"{cfg}: host enqueue {1e3 * (t1 - t0) / steps:.4f} ms/step, device {1e3 * (t2 - t0) / steps:.4f} ms/step",
                  flush=True)
        bench.release_workload(W)


if __name__ == "__main__":
    main()
