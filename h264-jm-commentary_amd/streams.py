"""streams.py — the multi-GPU execution model of the hot path: one independent P-picture stream
per rank (streams/GOPs are independent; no collective in the data path).

A "stream" holds a device-resident source sequence (an IDR picture and F P pictures, SURVEY.md
§8d's synthetic sequence) and encodes P pictures back to back, each one referencing the previous
picture's reconstruction (JM's IPPP with one reference frame):

    step i:  set_reference_slot(-2)     -- previous deblocked picture -> reference
             encode_slot(1 + i % F, P)  -- the whole macroblock wavefront of one picture, with
                                           DeblockFrame fused into it (jmh_frame_params.deblock)

With ``deblock=None`` the stream skips the loop filter and references the unfiltered
reconstruction (slot -1), which is what the oracle-backed stand-in of the CPU tests supports.

``timed_run`` times exactly ``steps`` steps in steady state.  The device pipelines pictures
(picture q runs diagonal d once picture q-1 is PIPE_LAG diagonals ahead), and a step only issues
the launches that bring its picture in, so after the warmup (at least ``depth`` steps: the fill)
every step retires exactly one picture.  The timed region is bracketed on both sides by a
barrier and a wait for every issued launch (``wait_issued``) — which does not drain the pictures
in flight — so it starts and ends with a full pipeline and holds exactly ``steps`` pictures of
work, independent of ``steps``.  The maximum wall time over ranks is returned (torch.distributed
with the process group the caller initialised; gloo is enough — only timings are reduced, never
picture data).

The encoder object only needs load_frame / encode_slot / set_reference_slot / wait_issued / sync
and ``depth``: the HIP encoder (jmhip.Encoder) in bench.py, an oracle-backed stand-in in the CPU
tests.
"""
import time

P_SLICE, I_SLICE = 0, 2


class PStream:
    def __init__(self, encoder, frames, qp, deblock=(0, 0, 0)):
        """frames: (y, u, v) pictures: [0] the IDR picture, [1:] the P pictures, cycled.
        deblock: (disable_idc, alpha_div2, beta_div2) of the device loop filter, or None."""
        assert len(frames) >= 2
        self.enc, self.qp, self.deblock = encoder, qp, deblock
        self.nseq = len(frames) - 1
        self.ref_slot = -1 if deblock is None else -2
        self.slots_used = []                              # slot per P step, in order (tests replay it)
        for i, f in enumerate(frames):
            encoder.load_frame(i, *f)
        self._encode(0, I_SLICE)                          # IDR picture -> first reference
        encoder.sync()

    def _encode(self, slot, slice_type):
        if self.deblock is None:
            self.enc.encode_slot(slot, slice_type, self.qp)
        else:
            self.enc.encode_slot(slot, slice_type, self.qp, deblock=self.deblock)

    def step(self, i):
        slot = 1 + i % self.nseq
        self.enc.set_reference_slot(self.ref_slot)        # previous (deblocked) picture -> reference
        self._encode(slot, P_SLICE)
        self.slots_used.append(slot)


def _max_over_ranks(dist, x):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_run(stream, steps, warmup, dist=None, on_start=None):
    """Run max(warmup, depth) untimed steps (the warmup, which also fills the pipeline), then
    exactly `steps` timed steps; returns the maximum seconds over ranks.  on_start() runs after
    the warmup's launches have completed (e.g. to reset the encoder's event sums).  Sets
    stream.warmup_steps to the number of untimed steps run."""
    enc = stream.enc
    prime = max(warmup, getattr(enc, "depth", 1))
    for i in range(prime):
        stream.step(i)
    enc.wait_issued()
    if on_start is not None:
        on_start()
    if dist is not None:
        dist.barrier()
    enc.wait_issued()
    t0 = time.perf_counter()
    for i in range(steps):
        stream.step(prime + i)
    enc.wait_issued()
    dt = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    stream.warmup_steps = prime
    return _max_over_ranks(dist, dt)
