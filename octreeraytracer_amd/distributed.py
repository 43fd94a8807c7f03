"""Multi-GPU frame partition and assembly.

The reference renders on one GL context; here one process drives one GPU
(torch.distributed, backend "nccl" = RCCL over xGMI).  The frame is cut into BAND-row bands
dealt round-robin to the ranks (rank r renders bands r, r+N, r+2N, ...), which balances
cheap sky rows against geometry rows.  Every rank renders the same number of rows (the
last bands of some ranks fall below the frame and come back as zeros), so the only
exchange -- gathering the bands to rank 0 -- is one equal-sized RCCL gather, followed by a
de-interleave into the final frame on rank 0.  Pixels are independent and the RNG is
seeded from the global pixel coordinate, so the assembled frame is
bit-identical to a single-GPU render.
"""
from __future__ import annotations

from .renderer import Tile

BAND = 16


def bands_per_rank(height: int, world: int, band: int = BAND) -> int:
    nbands = -(-height // band)
    return -(-nbands // world)


def rank_tile(width: int, height: int, rank: int, world: int, band: int = BAND) -> Tile:
    if world == 1:
        return Tile(0, width, 0, height)
    per = bands_per_rank(height, world, band)
    return Tile(0, width, rank * band, per * band, band, band * world)


def assemble(gathered, height: int, world: int, band: int = BAND, out=None):
    """gathered: [world, per*band, W, 3] (torch tensor or numpy array) -> [height, W, 3].
    Global band b*world + r is band b of rank r."""
    if world == 1:
        frame = gathered[0][:height]
        if out is not None:
            out[...] = frame
            return out
        return frame
    per = gathered.shape[1] // band
    W = gathered.shape[2]
    if hasattr(gathered, "permute"):
        g = gathered.reshape(world, per, band, W, 3).permute(1, 0, 2, 3, 4).reshape(per * world * band, W, 3)
    else:
        g = gathered.reshape(world, per, band, W, 3).transpose(1, 0, 2, 3, 4).reshape(per * world * band, W, 3)
    if out is not None:
        if hasattr(out, "copy_"):
            out.copy_(g[:height])
        else:
            out[...] = g[:height]
        return out
    return g[:height]


class GatherTimeout(RuntimeError):
    """A frame's band gather did not complete within FrameGather's bound."""

    def __init__(self, rank: int, slot: int, timeout_s: float, why: str = ""):
        super().__init__(f"rank {rank}: the band gather of slot {slot} did not complete within {timeout_s} s"
                         + (f" ({why.splitlines()[0][:200]})" if why else ""))
        self.rank, self.slot = rank, slot


class FrameGather:
    """Gather every rank's band tile to rank 0 and assemble the frame (torch.distributed).

    __call__ is synchronous.  submit()/finish() pipeline frames: submit issues the gather of a
    tile asynchronously into receive slot `slot` (depth slots), finish waits for it (a stream
    wait for RCCL, no host block) and assembles the frame on rank 0 -- so frame k's gather
    and assembly overlap frame k+1's render.  A rank must not overwrite a submitted tile
    before finish() of that submission (bench.py double-buffers its tiles)."""

    def __init__(self, dist, width: int, height: int, world: int, rank: int, device, band: int = BAND,
                 depth: int = 1, timeout_s: float | None = None):
        """timeout_s: bound of finish()'s wait for a gather (None: the process group's own); on
        expiry finish() raises GatherTimeout naming the rank and the slot.  (With the nccl
        backend an async gather's wait only orders the streams: a stalled RCCL gather is
        bounded by the process group's timeout, init_process_group(timeout=...), whose
        watchdog aborts the process.)"""
        import torch
        self.dist, self.world, self.rank, self.height, self.band = dist, world, rank, height, band
        self.timeout_s = timeout_s
        rows = rank_tile(width, height, rank, world, band).rows
        self.slots = [torch.empty((world, rows, width, 3), dtype=torch.float32, device=device)
                      for _ in range(depth)] if rank == 0 and world > 1 else None
        self.gathered = self.slots[0] if self.slots else None
        self.frame = torch.empty((height, width, 3), dtype=torch.float32, device=device) if rank == 0 else None

    def __call__(self, local):
        if self.world == 1:
            return local
        self.dist.gather(local, list(self.gathered.unbind(0)) if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            assemble(self.gathered, self.height, self.world, self.band, out=self.frame)
            return self.frame
        return None

    def submit(self, local, slot: int = 0):
        """Start gathering `local` (async); returns a handle for finish()."""
        if self.world == 1:
            return (None, slot, local)
        dst = list(self.slots[slot].unbind(0)) if self.rank == 0 else None
        return (self.dist.gather(local, dst, dst=0, async_op=True), slot, local)

    def finish(self, handle):
        """Complete a submit(): returns the assembled frame on rank 0 (None elsewhere)."""
        work, slot, local = handle
        if self.world == 1:
            return local[:self.height]  # nothing to gather: the tile is the frame
        if self.timeout_s is None:
            work.wait()
        else:
            from datetime import timedelta
            try:
                ok = work.wait(timeout=timedelta(seconds=self.timeout_s))
            except RuntimeError as e:  # gloo raises on expiry
                raise GatherTimeout(self.rank, slot, self.timeout_s, str(e)) from e
            if ok is False:
                raise GatherTimeout(self.rank, slot, self.timeout_s, "wait returned False")
        if self.rank == 0:
            assemble(self.slots[slot], self.height, self.world, self.band, out=self.frame)
            return self.frame
        return None
