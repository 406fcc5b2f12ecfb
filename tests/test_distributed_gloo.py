"""The N>1 path (partition -> per-rank tile -> one gather -> de-interleave) with
world_size 2 and 3 on the gloo backend (CPU).  Each rank renders its tile
with the oracle's kernel-mode restatement (the bit-exact CPU twin of the HIP
kernel), so the assembled frame must equal the single-process frame bit for
bit -- the same property bench.py relies on over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, SEED = 48, 29, 2, 77


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, row_block, outdir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "ray-tracing-in-one-weekend_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import rtow
    import rtow_dist
    import oracle_lib
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=W / H)

    def render_tile(p):
        out, _ = oracle_lib.kernel_render(scene, cam, p, threads=2)
        return torch.from_numpy(out)

    frame = rtow_dist.render_distributed(render_tile, W, H, SPP, world, rank, row_block=row_block,
                                         seed=SEED)
    if rank == 0:
        np.save(os.path.join(outdir, f"frame_{world}_{row_block}.npy"), frame)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,row_block", [(2, 8), (3, 4)])
def test_gloo_distributed_frame_equals_single_process(rtow, oracle, tmp_path, world, row_block):
    mp.spawn(_worker, args=(world, _free_port(), row_block, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / f"frame_{world}_{row_block}.npy")
    full, _ = oracle.kernel_render(rtow.final_scene(), rtow.camera_cpu(aspect=W / H),
                                   rtow.make_params(W, H, SPP, seed=SEED))
    assert got.shape == (H, W, 3)
    assert np.array_equal(got, full)


def test_assemble_inverts_partition(rtow):
    import rtow_dist
    rng = np.random.default_rng(1)
    frame = rng.random((37, 5, 3)).astype(np.float32)
    for world in (1, 2, 4, 8):
        tiles = []
        for r in range(world):
            p = rtow_dist.partition(5, 37, 1, world, r, row_block=4)
            rows = rtow.local_to_global_rows(p)
            t = np.zeros((p.local_rows, 5, 3), np.float32)
            t[rows < 37] = frame[rows[rows < 37]]
            tiles.append(t)
        assert np.array_equal(rtow_dist.assemble(np.stack(tiles), 37, world, row_block=4), frame)
