"""Batched record types mirroring the fields of Mitsuba's records that the
sunsky emitter reads or writes (include/mitsuba/render/records.h:20-145,
interaction.h).  Vectors are SoA torch tensors of shape (3, n) -- the layout
Dr.Jit uses for Vector3f in the JIT variants; spectral wavelengths are (k, n)."""
from dataclasses import dataclass, field
from typing import Optional

import torch


@dataclass
class SurfaceInteraction3f:
    wi: Optional[torch.Tensor] = None            # (3, n) incident direction (si.wi)
    wavelengths: Optional[torch.Tensor] = None   # (k, n) spectral variants


@dataclass
class Interaction3f:
    p: Optional[torch.Tensor] = None             # (3, n) reference point; None = origin
    time: Optional[torch.Tensor] = None
    wavelengths: Optional[torch.Tensor] = None   # (k, n) spectral variants


@dataclass
class DirectionSample3f:
    p: Optional[torch.Tensor] = None
    n: Optional[torch.Tensor] = None
    uv: Optional[torch.Tensor] = None
    time: Optional[torch.Tensor] = None
    pdf: Optional[torch.Tensor] = None
    delta: bool = False
    d: Optional[torch.Tensor] = None
    dist: Optional[torch.Tensor] = None
    emitter: object = None


@dataclass
class Ray3f:
    o: Optional[torch.Tensor] = None
    d: Optional[torch.Tensor] = None
    time: Optional[torch.Tensor] = None
    wavelengths: Optional[torch.Tensor] = None


@dataclass
class ScalarBoundingBox3f:
    min: tuple = field(default_factory=lambda: (float("inf"),) * 3)
    max: tuple = field(default_factory=lambda: (float("-inf"),) * 3)

    def valid(self):
        return all(a <= b for a, b in zip(self.min, self.max))
