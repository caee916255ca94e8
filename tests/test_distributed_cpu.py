"""The multi-GPU data path on CPU: gloo, world size 2 (and 3). Each rank renders its
interleaved rows with the CPU oracle (stand-in for the device render, same row semantics),
FrameGather assembles the frame on rank 0, and it must equal a single full render bitwise."""
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
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, spp, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import golden_io as G
        import oracle_binding as O
        from raytracinginoneweekend_amd.rowtiles import FrameGather, rank_params
        s, m = G.scene("huge")
        p = rank_params(W, H, spp, world, rank, seed=77)
        tile_np, _ = O.render_f32(s, m, O.camera_default(W, H), p, threads=2)
        tile = torch.from_numpy(tile_np)
        g = FrameGather(tile, world, rank)
        frame = g(tile)
        if rank == 0:
            np.save(out_path, frame.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_row_tiles_gather_bitwise(tmp_path, world):
    W, H, spp = 48, 24, 2
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, spp, out), nprocs=world, join=True,
                       start_method="spawn")
    frame = np.load(out)
    import golden_io as G
    import oracle_binding as O
    s, m = G.scene("huge")
    whole, _ = O.render_f32(s, m, O.camera_default(W, H), O.make_params(W, H, spp, seed=77))
    np.testing.assert_array_equal(frame.view(np.uint32), whole.view(np.uint32))


def test_rank_rows_requires_divisible_height():
    from raytracinginoneweekend_amd.rowtiles import rank_rows
    assert rank_rows(720, 8, 3) == (3, 8, 90)
    with pytest.raises(ValueError):
        rank_rows(721, 8, 0)
