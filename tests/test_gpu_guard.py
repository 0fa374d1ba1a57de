"""NaN guard bands in the default GPU suite (SURVEY.md section 5's "poison
halo" debug mode).

With ROMS_GPU_GUARD=1 (read by every roms_gpu_init) each field and scratch
array is allocated with 4096 NaN-filled doubles on both sides, so a kernel
that reads outside an array (a stencil that steps past a halo, a segment
solver's clamped level, a pack index off the strip) pulls a NaN into the
result.  The decomposition, drop-in and cross-process IPC tests then run
unchanged and must still be bitwise equal to their references.
"""
import pytest

import test_gpu_dropin as dropin
import test_gpu_ipc as ipc
import test_gpu_multirank as mr

pytestmark = pytest.mark.gpu


@pytest.fixture
def guard(monkeypatch):
    monkeypatch.setenv("ROMS_GPU_GUARD", "1")


@pytest.mark.parametrize("kind", ["filament", "basin_lmd", "pipes"])
@pytest.mark.parametrize("npx,npe", [(2, 2), (3, 2)])
def test_guard_decomposition_bitwise(kind, npx, npe, guard):
    mr.check_decomposition(mr._case(kind), npx, npe)


def test_guard_uneven_split(guard, monkeypatch):
    mr.test_fast_loop_interval_fits_uneven_split("basin", 81, 8, "4", 2, monkeypatch)


def test_guard_dropin_c3_switch_set(guard):
    dropin._single_rank(dropin.c3_cfg(), 6)


def test_guard_dropin_iceland_switch_set(guard):
    dropin._single_rank(dropin.c4_cfg(L=48, sponge=1.0e3, island=1), 6)


def test_guard_dropin_c1_2x2(guard):
    dropin.test_dropin_sequence_c1_filament_128_2x2()


@pytest.mark.parametrize("kind", ["filament", "basin_obc"])
def test_guard_ipc_processes(kind, guard):
    ipc._ranks(kind, 2, 2)
