"""Benchmark / parity configurations (BASELINE.json `configs`, SURVEY.md §8 dims table)."""
from __future__ import annotations

from dataclasses import dataclass

POC, SOC = 0, 1


@dataclass(frozen=True)
class Config:
    name: str
    n: int
    m: int
    k: int
    cones: tuple  # ((kind, offs, dim), ...)
    batch: int
    fixed_k: int  # headline fixed-iteration count
    config_id: int

    @property
    def seed(self) -> int:
        return 0x534F4350 + self.config_id  # "SOCP" + config id


C0B = Config("C0b", 10, 8, 3, ((SOC, 0, 3),), 1, 5, 0)
C1 = Config("C1", 32, 8, 48, ((SOC, 0, 48),), 4096, 3, 1)
C2 = Config("C2", 64, 16, 96, ((POC, 0, 32), (SOC, 32, 32), (SOC, 64, 32)), 65536, 8, 2)
C3 = Config("C3", 64, 16, 96, ((POC, 0, 32), (SOC, 32, 32), (SOC, 64, 32)), 524288, 8, 2)
C4 = Config("C4", 512, 64, 640, tuple((SOC, 80 * i, 80) for i in range(8)), 1024, 5, 4)

CONFIGS = {c.name: c for c in (C0B, C1, C2, C3, C4)}
