"""The multi-GPU data path on CPU: gloo, world sizes 1-4. Each rank renders its interleaved
rows with the CPU oracle (stand-in for the device render, same row semantics), FrameGather
assembles the frame on rank 0, and it must equal a single full render bitwise: f32 tiles, u8
tiles (the gamma epilogue on each rank before the gather, bench.py --output rgb8), and ragged
heights (H not a multiple of the world size: the first H mod N ranks hold one row more)."""
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


def _worker(rank, world, port, W, H, spp, out_path, u8=False):
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
        if u8:
            tile_np = O.epilogue_rgb8(tile_np)
        tile = torch.from_numpy(tile_np)
        g = FrameGather(tile, world, rank, height=H)
        frame = g(tile)
        if rank == 0:
            np.save(out_path, frame.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,u8", [(1, 24, False), (2, 24, False), (3, 24, False), (2, 24, True),
                                        (3, 25, False), (2, 23, True), (4, 26, False), (4, 27, True)])
def test_row_tiles_gather_bitwise(tmp_path, world, H, u8):
    W, spp = 48, 2
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, spp, out, u8), nprocs=world, join=True,
                       start_method="spawn")
    frame = np.load(out)
    import golden_io as G
    import oracle_binding as O
    s, m = G.scene("huge")
    whole, _ = O.render_f32(s, m, O.camera_default(W, H), O.make_params(W, H, spp, seed=77))
    if u8:
        assert frame.dtype == np.uint8
        np.testing.assert_array_equal(frame, O.epilogue_rgb8(whole))
    else:
        np.testing.assert_array_equal(frame.view(np.uint32), whole.view(np.uint32))


def test_rank_rows_ragged():
    from raytracinginoneweekend_amd.rowtiles import rank_params, rank_rows
    assert rank_rows(720, 8, 3) == (3, 8, 90)
    assert [rank_rows(721, 8, r)[2] for r in range(8)] == [91] + [90] * 7
    assert sum(rank_rows(2159, 8, r)[2] for r in range(8)) == 2159
    with pytest.raises(ValueError):
        rank_params(8, 3, 1, 4, 3)  # rank 3 of 4 has no row of a 3-row frame
    with pytest.raises(ValueError):
        rank_rows(720, 8, 8)
