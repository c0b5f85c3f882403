"""Drop-in binding (CPU, no device calls): zero-argument constructors read the reference's
``quadruped_pympc.config`` when that package is installed, and ``device_id='auto'`` maps replica
processes onto GPUs (SURVEY 8(b) construction, 8(e) replica mode)."""
import multiprocessing as mp
import sys
import types

import numpy as np
import pytest

from quadruped_pympc_amd import config as mirror
from quadruped_pympc_amd import runtime


@pytest.fixture
def fake_reference(monkeypatch):
    """A stand-in ``quadruped_pympc`` package whose config names HyQReal (the mirror's robot is aliengo)."""
    pkg = types.ModuleType("quadruped_pympc")
    pkg.__path__ = []  # a package
    cfg = types.ModuleType("quadruped_pympc.config")
    cfg.robot = "hyqreal1"
    cfg.mass, inertia = mirror.ROBOTS["hyqreal1"]
    cfg.inertia = np.array(inertia)
    cfg.hip_height = 0.5
    cfg.gravity_constant = 9.81
    cfg.mpc_params = dict(mirror.mpc_params)
    cfg.mpc_params.update(num_parallel_computations=2048, horizon=12, sampling_method="mppi",
                          control_parametrization="zero_order", grf_max=cfg.mass * 9.81)
    cfg.mpc_params.pop("device_id", None)  # the reference's config has no device_id key
    cfg.simulation_params = dict(mirror.simulation_params)
    pkg.config = cfg
    monkeypatch.setitem(sys.modules, "quadruped_pympc", pkg)
    monkeypatch.setitem(sys.modules, "quadruped_pympc.config", cfg)
    return cfg


def test_zero_arg_constructors_bind_the_reference_config(fake_reference):
    from quadruped_pympc_amd.controllers.sampling.centroidal_nmpc_hip import Sampling_MPC
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import VisualFootholdAdaptation
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface

    assert runtime.active_config() is fake_reference
    mpc = Sampling_MPC()  # construction is lazy: no HIP call
    assert mpc.mass == fake_reference.mass and mpc.num_parallel_computations == 2048
    np.testing.assert_array_equal(mpc.inertia, np.asarray(fake_reference.inertia, np.float32))
    assert mpc.device_id == "auto"
    iface = SRBDControllerInterface()
    assert iface.controller.mass == fake_reference.mass
    vfa = VisualFootholdAdaptation(("FL", "FR", "RL", "RR"), adaptation_strategy="height")
    assert vfa._device_id == "auto"


def test_mirror_when_reference_absent(monkeypatch):
    monkeypatch.delitem(sys.modules, "quadruped_pympc", raising=False)
    monkeypatch.delitem(sys.modules, "quadruped_pympc.config", raising=False)
    assert runtime.active_config() is mirror
    from quadruped_pympc_amd.controllers.sampling.centroidal_nmpc_hip import Sampling_MPC

    assert Sampling_MPC().mass == mirror.mass


def test_broken_reference_config_raises(monkeypatch):
    """Installed but unimportable (e.g. gym_quadruped missing): raise, never fall back silently."""
    pkg = types.ModuleType("quadruped_pympc")
    pkg.__path__ = []
    monkeypatch.setitem(sys.modules, "quadruped_pympc", pkg)
    monkeypatch.delitem(sys.modules, "quadruped_pympc.config", raising=False)
    with pytest.raises(ImportError):
        runtime.active_config()


def test_explicit_ordinal_and_auto(monkeypatch):
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.delenv("SRBD_REPLICA_INDEX", raising=False)
    assert runtime.resolve_device_id(3, device_count=8) == 3
    assert runtime.resolve_device_id("2", device_count=8) == 2
    assert runtime.resolve_device_id("auto", device_count=8) == 0  # main process
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert runtime.resolve_device_id("auto", device_count=4) == 1
    assert runtime.resolve_device_id(None, device_count=0) == 0
    # an explicit replica index (a launcher's) wins over LOCAL_RANK and the multiprocessing identity
    monkeypatch.setenv("SRBD_REPLICA_INDEX", "6")
    assert runtime.replica_source() == (6, "SRBD_REPLICA_INDEX")
    assert runtime.resolve_device_id("auto", device_count=4) == 2


def test_auto_resolution_is_logged(monkeypatch, caplog):
    import logging

    monkeypatch.setenv("SRBD_REPLICA_INDEX", "3")
    with caplog.at_level(logging.INFO, logger="quadruped_pympc_amd.runtime"):
        assert runtime.resolve_device_id("auto", device_count=2) == 1
    assert "GPU 1" in caplog.text and "SRBD_REPLICA_INDEX" in caplog.text


def _child(q):
    import os

    os.environ.pop("LOCAL_RANK", None)
    os.environ.pop("SRBD_REPLICA_INDEX", None)
    q.put(runtime.resolve_device_id("auto", device_count=8))


def test_replica_processes_spread_over_gpus():
    """batched_simulations.py:43-55: one Process per replica -> distinct GPUs (i mod G)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_child, args=(q,)) for _ in range(4)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(60)
    assert len(set(got)) == 4, got
