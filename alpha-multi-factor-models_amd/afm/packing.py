"""Persistent send buffers for the packed all-gathers of the multi-rank step.

A step's exchange of several small per-rank tensors goes out as ONE all-gather of their bytes.
``Comm.all_gather_packed`` builds that byte vector each call (a pad / fill and a copy per part,
then a concatenation: launches on the exchange's critical path); a ``SendBuffer`` is allocated
once, its parts are typed views at 8-byte-aligned offsets that keep their fill value (NaN or 0)
wherever a step does not write, and a step only copies its live rows in before
``comm.all_gather_buffer(sb)``, which returns the gathered parts as ``[world, *shape]`` views of
the received bytes (no copy)."""
from __future__ import annotations


class SendBuffer:
    def __init__(self, specs, device):
        """specs: [(shape, dtype, fill)] -- one typed part each, filled once here."""
        import torch
        self.layout, off = [], 0
        for shape, dtype, _ in specs:
            n = torch.Size(shape).numel() * torch.empty((), dtype=dtype).element_size()
            self.layout.append((off, n, dtype, tuple(shape)))
            off += (n + 7) // 8 * 8
        self.buf = torch.empty(max(off, 8), dtype=torch.uint8, device=device)
        self.parts = []
        for (o, n, dtype, shape), (_, _, fill) in zip(self.layout, specs):
            p = self.buf[o:o + n].view(dtype).view(shape)
            p.fill_(fill)
            self.parts.append(p)


def unpack_gathered(g, layout, world: int):
    """The typed ``[world, *shape]`` views of the parts of a gathered byte buffer ``g``
    ([world, nbytes]); every offset and the row length are 8-byte multiples, so each part is a
    strided view (no copy)."""
    return [g[:, o:o + n].view(dtype).view((world,) + shape) for o, n, dtype, shape in layout]
