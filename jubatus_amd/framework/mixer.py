"""Mixer interface, dummy mixer and factory (reference C22:
jubatus/server/framework/mixer/{mixer.hpp,dummy_mixer.hpp,mixer_factory.cpp}).

``create_mixer`` chooses by the ``--mixer`` string: linear_mixer (RCCL
all-reduce MIX, parallel/linear_mixer.py), random_mixer / broadcast_mixer /
skip_mixer (pairwise send/recv schedules, parallel/push_mixer.py); anything
else raises. Standalone servers get a DummyMixer whose methods are no-ops
(the reference never starts the mixer in standalone mode,
server_helper.hpp:240-243).
"""
from __future__ import annotations

from typing import Any


class UnsupportedMixables(RuntimeError):
    pass


class Mixer:
    def register_api(self, rpc) -> None: ...
    def set_driver(self, driver) -> None: ...
    def start(self) -> None: ...
    def stop(self) -> None: ...
    def updated(self, n: int = 1) -> None: ...
    def get_status(self, status: dict[str, str]) -> None: ...
    def type(self) -> str: return "mixer"
    def do_mix(self) -> bool: return False


class DummyMixer(Mixer):
    def __init__(self):
        self.driver = None
        self.count = 0

    def set_driver(self, driver) -> None:
        self.driver = driver

    def updated(self, n: int = 1) -> None:
        self.count += n

    def type(self) -> str:
        return "dummy_mixer"


MIXERS = ("linear_mixer", "random_mixer", "broadcast_mixer", "skip_mixer")


def create_mixer(argv, coord, rw_mutex, server_type: str, protocol_version: int = 1,
                 backend: str | None = None) -> Mixer:
    if argv.is_standalone():
        return DummyMixer()
    name = argv.mixer
    if name == "linear_mixer":
        from ..parallel.linear_mixer import LinearMixer
        return LinearMixer(argv, coord, rw_mutex, server_type, protocol_version, backend)
    if name in ("random_mixer", "broadcast_mixer", "skip_mixer"):
        from ..parallel.push_mixer import PushMixer
        return PushMixer(name, argv, coord, rw_mutex, server_type, protocol_version, backend)
    raise ValueError(f"unknown mixer: {name}")


def describe(m: Any) -> str:
    return m.type() if isinstance(m, Mixer) else type(m).__name__
