"""streams.py — the multi-GPU execution model of the hot path: one independent P-picture stream
per rank (streams/GOPs are independent; no collective in the data path).

A "stream" holds two device-resident source pictures and encodes P pictures back to back, each
one referencing the previous picture's reconstruction (JM's IPPP with one reference frame):

    step i:  set_reference_slot(-1)     -- previous reconstruction -> reference (+ qpel planes)
             encode_slot(1 + i % 2, P)  -- the whole macroblock wavefront of one picture

``timed_run`` brackets exactly ``steps`` steps with barrier + device sync on both sides and
returns the maximum wall time over ranks (torch.distributed with the process group the caller
initialised; gloo is enough — only the timing is reduced, never picture data).

The encoder object only needs load_frame / encode_slot / set_reference_slot / sync: the HIP
encoder (jmhip.Encoder) in bench.py, an oracle-backed stand-in in the CPU tests.
"""
import time

P_SLICE, I_SLICE = 0, 2


class PStream:
    def __init__(self, encoder, frames, qp):
        """frames: three (y, u, v) pictures: [0] the IDR picture, [1], [2] alternate as P pictures."""
        self.enc, self.qp = encoder, qp
        for i, f in enumerate(frames[:3]):
            encoder.load_frame(i, *f)
        encoder.encode_slot(0, I_SLICE, qp)               # IDR picture -> first reference
        encoder.sync()

    def step(self, i):
        self.enc.set_reference_slot(-1)                   # previous reconstruction -> reference
        self.enc.encode_slot(1 + (i % 2), P_SLICE, self.qp)


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
