"""Single-GPU rehearsal of the N > 1 bench step inside a hipGraph, with a real RCCL all-reduce.

bench.py captures the multi-rank step (band apply + interface pack + RCCL all-reduce + unpack) in
hipGraphs.  RCCL refuses two ranks on one GPU, so this runs a one-rank "nccl" process group on the
left strip of a 128 x 64-element, P=8 mesh split in two (bounds [0, 64, 128]): the strip has a
right interface line, the pack / all-reduce / unpack kernels all run, and a one-rank all-reduce
leaves the buffer as it is.  Checks that the graph replay gives the eager step's bits and prints
the per-step time of both, and of the apply alone.

Run:  python tools/rccl_graph_check.py   (one GPU)
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import bench
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    from sem_amd.parallel import StripPartition

    P, ne, Pe = 8, 64, 40.0
    part = StripPartition(2 * ne, 2)
    mesh = get_mesh(P, 2 * ne, ne, 1.0 / ne, 1.0 / ne, 0, ne, 0)
    T, u, v = bench.make_inputs(mesh)
    y = torch.empty_like(T)
    kw = dict(c_stiff=1.0, c_gradx=Pe, cu=u, c_grady=Pe, cv=v, dir_mode=_lib.DIR_IDENTITY,
              dir_sides=_lib.SIDE_W | _lib.SIDE_E)
    exch = part.exchanger(mesh, dist, kind="allreduce")

    def step():
        mesh.apply(T, y, **kw)
        exch(y)

    step()
    torch.cuda.synchronize()
    y_eager = y.clone()
    out = {}
    for name, fn, graph in (("apply_only_graph", lambda: mesh.apply(T, y, **kw), True),
                            ("step_eager", step, False), ("step_graph", step, True)):
        y.zero_()
        secs, wall = bench.time_steps(fn, 1000, 100, dev, use_graph=graph, dist=dist)
        out[name + "_us"] = secs / 1000 * 1e6
        out[name + "_host_us"] = wall / 1000 * 1e6
    out["graph_bitwise_equal_eager"] = bool(torch.equal(y, y_eager))
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    if not out["graph_bitwise_equal_eager"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
