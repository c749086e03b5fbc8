"""world_size-2 gloo run of the multi-GPU sharding (distributed.py) on CPU.

Each rank traces its sample range of every pixel with the CPU build of the kernel's own code
(tests/hostcheck standing in for rt_trace_device), gloo reduces the float64 sums to rank 0, and the
reduced mean must equal the single-process render up to the order of the partial-sum additions."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import golden_cases as gc
    import hostcheck_binding as hb
    from blenderraytracer_amd.distributed import ShardedRender

    rt, c = gc.tracer_for(case)
    packed = rt.packed()

    def cpu_trace(buf, settings):
        r = hb.render(packed, settings)
        buf.copy_(torch.from_numpy((r["mean"] * settings.samples).reshape(-1)))

    job = ShardedRender(rt, rank=rank, world=world, device=torch.device("cpu"), trace_fn=cpu_trace)
    job.step()
    if rank == 0:
        np.save(out_path, job.sum.numpy())
        np.save(out_path + ".range.npy", np.array(job.range))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("kitchen_sink", 2), ("rtow_small", 2), ("cornell_small", 3)])
def test_sharded_render_gloo(tmp_path, case, world):
    import golden_cases as gc
    import hostcheck_binding as hb
    hb.build()
    out = str(tmp_path / "sum.npy")
    mp.start_processes(_worker, args=(world, _free_port(), case, out), nprocs=world, start_method="spawn", join=True)
    reduced = np.load(out).reshape(-1, 3)
    rt, c = gc.tracer_for(case)
    full = hb.render(rt.packed(), rt.settings())
    expect = (full["mean"] * rt.settings().samples).reshape(-1, 3)
    assert np.allclose(reduced, expect, rtol=1e-13, atol=1e-15)
    # and the reduced mean matches the reference fixture (full-frame cases only)
    if c["crop"] == [0, 0, c["width"], c["height"]]:
        lin = gc.load_array(case, "linear").reshape(-1, 3)
        assert np.allclose(reduced / rt.settings().samples, lin, rtol=1e-12, atol=1e-15, equal_nan=True)


def test_sample_ranges_partition():
    from blenderraytracer_amd.distributed import sample_range
    for S in (1, 7, 64, 512, 1024):
        for N in (1, 2, 3, 4, 8):
            rs = [sample_range(r, N, S) for r in range(N)]
            assert rs[0][0] == 0 and rs[-1][1] == S
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
