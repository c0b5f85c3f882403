"""Minimal ``LegsAttr`` (the reference imports it from the absent ``gym_quadruped``).

Attribute and item access by leg name (FL, FR, RL, RR), iteration in leg order,
as used by srbd_controller_interface.py and visual_foothold_adaptation.py.
"""
from __future__ import annotations

LEG_NAMES = ("FL", "FR", "RL", "RR")


class LegsAttr:
    __slots__ = LEG_NAMES

    def __init__(self, FL=None, FR=None, RL=None, RR=None):
        self.FL, self.FR, self.RL, self.RR = FL, FR, RL, RR

    def __getitem__(self, key):
        if isinstance(key, int):
            key = LEG_NAMES[key]
        return getattr(self, key)

    def __setitem__(self, key, value):
        if isinstance(key, int):
            key = LEG_NAMES[key]
        setattr(self, key, value)

    def __iter__(self):
        return iter([self.FL, self.FR, self.RL, self.RR])

    def to_list(self, order=LEG_NAMES):
        return [getattr(self, k) for k in order]

    def __repr__(self):
        return f"LegsAttr(FL={self.FL!r}, FR={self.FR!r}, RL={self.RL!r}, RR={self.RR!r})"
