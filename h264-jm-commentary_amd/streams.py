"""streams.py — the multi-GPU execution model of the hot path: one independent P-picture stream
per rank (streams/GOPs are independent; no collective in the data path).

A "stream" holds two device-resident source pictures and encodes P pictures back to back, each
one referencing the previous picture's reconstruction (JM's IPPP with one reference frame):

    step i:  set_reference_slot(-2)     -- previous deblocked picture -> reference (+ qpel planes)
             encode_slot(1 + i % 2, P)  -- the whole macroblock wavefront of one picture, with
                                           DeblockFrame fused into it (jmh_frame_params.deblock)

With ``deblock=None`` the stream skips the loop filter and references the unfiltered
reconstruction (slot -1), which is what the oracle-backed stand-in of the CPU tests supports.

``timed_run`` brackets exactly ``steps`` steps with barrier + device sync on both sides and
returns the maximum wall time over ranks (torch.distributed with the process group the caller
initialised; gloo is enough — only the timing is reduced, never picture data).

The encoder object only needs load_frame / encode_slot / set_reference_slot / sync: the HIP
encoder (jmhip.Encoder) in bench.py, an oracle-backed stand-in in the CPU tests.
"""
import time

P_SLICE, I_SLICE = 0, 2


class PStream:
    def __init__(self, encoder, frames, qp, deblock=(0, 0, 0)):
        """frames: three (y, u, v) pictures: [0] the IDR picture, [1], [2] alternate as P pictures.
        deblock: (disable_idc, alpha_div2, beta_div2) of the device loop filter, or None."""
        self.enc, self.qp, self.deblock = encoder, qp, deblock
        self.ref_slot = -1 if deblock is None else -2
        for i, f in enumerate(frames[:3]):
            encoder.load_frame(i, *f)
        self._encode(0, I_SLICE)                          # IDR picture -> first reference
        encoder.sync()

    def _encode(self, slot, slice_type):
        if self.deblock is None:
            self.enc.encode_slot(slot, slice_type, self.qp)
        else:
            self.enc.encode_slot(slot, slice_type, self.qp, deblock=self.deblock)

    def step(self, i):
        self.enc.set_reference_slot(self.ref_slot)        # previous (deblocked) picture -> reference
        self._encode(1 + (i % 2), P_SLICE)


def timed_run(stream, steps, warmup, dist=None, on_start=None):
    """Run warmup untimed steps, then exactly `steps` timed steps; max seconds over ranks.
    on_start() runs after the warmup has drained (e.g. to reset the encoder's event sums)."""
    for i in range(warmup):
        stream.step(i)
    stream.enc.sync()
    if on_start is not None:
        on_start()
    if dist is not None:
        dist.barrier()
    stream.enc.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        stream.step(warmup + i)
    stream.enc.sync()
    dt = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt
