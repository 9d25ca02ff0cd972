"""CPU tests of the oracle's constraint solvers (mj_fwdConstraint) and of the
pyramidal-cone regulariser (mj_makeImpedance), before they are trusted as the GPU's checker.

* PGS (dual), Newton and CG (primal) minimise the same convex problem: from one contact state the
  three give the same qacc once converged (PGS run to 20000 sweeps at tolerance 1e-15).
* `<option solver>` is honoured (Newton is MuJoCo's default), `ls_tolerance` / `ls_iterations` parse.
* Pyramid edges: R = 2 mu^2 / impratio * (1 - imp) / imp * tran (1 + mu^2) for every edge of a
  box resting on the floor, with impratio 1 and 4.
"""
from pathlib import Path

import numpy as np
import pytest

from conftest import ARM7, REF_SCENE
from mujoco_ros2_simulation_amd import sim, synth
import binding

ARM_BOXES = ARM7.parent / "arm_boxes.xml"


def with_option(path: Path, option: str) -> "sim.Model":
    xml = path.read_text().replace('solver="PGS" iterations="50"', option)
    return sim.Model.from_string(xml, str(path.parent))


def test_solver_option_parsed():
    assert sim.Model.load(REF_SCENE).solver == 2          # no <option solver>: Newton
    m = with_option(ARM_BOXES, 'solver="CG" iterations="7" ls_tolerance="0.05" ls_iterations="9"')
    assert (m.solver, m.iterations, m.ls_iterations) == (1, 7, 9)
    assert m.ls_tolerance == pytest.approx(0.05)
    assert sim.Model.load(ARM_BOXES).solver == 0
    with pytest.raises(sim.MrsError):
        with_option(ARM_BOXES, 'solver="PGS" impratio="0"')


def test_three_solvers_one_optimum():
    # a settled C5 state with ~30 contacts (~130 rows)
    m0 = sim.Model.load(ARM_BOXES)
    d = binding.OracleData(m0)
    d.qpos[:] = synth.initial_qpos(m0, np.arange(1))[0]
    d.step(60)
    q, v = d.qpos.copy(), d.qvel.copy()
    qacc = {}
    for name, opt in [("PGS", 'solver="PGS" iterations="20000" tolerance="1e-15"'),
                      ("Newton", 'solver="Newton" iterations="100"'),
                      ("CG", 'solver="CG" iterations="1000" tolerance="1e-15"')]:
        m = with_option(ARM_BOXES, opt)
        e = binding.OracleData(m)
        e.qpos[:] = q
        e.qvel[:] = v
        e.forward()
        assert e.nefc > 100
        qacc[name] = e.qacc.copy()
        if name == "Newton":
            assert e.solver_niter <= 10
    scale = np.maximum(np.abs(qacc["Newton"]), 1.0)
    # PGS stalls at ~1e-6 of the optimum on this 130-row problem (its sweep improvement underflows)
    assert np.max(np.abs(qacc["PGS"] - qacc["Newton"]) / scale) < 1e-5
    assert np.max(np.abs(qacc["CG"] - qacc["Newton"]) / scale) < 1e-4


@pytest.mark.parametrize("impratio", [1.0, 4.0])
def test_pyramid_edge_regulariser(impratio):
    xml = f"""<mujoco><option timestep="0.002" impratio="{impratio}" solver="Newton"/><worldbody>
      <geom type="plane" size="0 0 1" friction="0.7 0.005 0.0001"/>
      <body pos="0 0 0.0995"><freejoint/><geom type="box" size="0.1 0.1 0.1" mass="2" friction="0.4 0.005 0.0001"/></body>
    </worldbody></mujoco>"""
    m = sim.Model.from_string(xml)
    d = binding.OracleData(m)
    d.forward()
    efc = d.efc()
    assert d.ncon == 4 and len(efc["R"]) == 16
    mu = 0.7                                      # max of the two geoms' sliding friction
    tran = m.body_invweight0[1, 0]                # world body has zero invweight
    # default solimp (0.9, 0.95, 0.001, 0.5, 2) at penetration 0.0005 = half the width: imp midway
    x = 0.0005 / 0.001
    y = x ** 2 / 0.5 ** (2 - 1)
    imp = 0.9 + y * (0.95 - 0.9)
    want = 2 * mu * mu / impratio * (1 - imp) / imp * tran * (1 + mu * mu)
    np.testing.assert_allclose(efc["R"], want, rtol=1e-9)
