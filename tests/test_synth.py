"""Philox4x32-10 against the Random123 known-answer vectors and the synthetic-input contract."""
import numpy as np

from mujoco_ros2_simulation_amd import synth


def test_philox_kat():
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, out in cases:
        got = synth.philox4x32(np.array(ctr, dtype=np.uint32), key=key)
        assert tuple(int(x) for x in got) == out


def test_streams_depend_on_global_env_id(s2_model):
    a = synth.ctrl_table(s2_model, np.arange(0, 16), 5, 10)
    b = synth.ctrl_table(s2_model, np.arange(8, 16), 5, 10)
    np.testing.assert_array_equal(a[:, 8:], b)
    q = synth.initial_qpos(s2_model, np.arange(16))
    assert np.all(np.abs(q - s2_model.qpos0) <= 0.1)
