"""MJCF loader / writer: the compiled gripper written as MJCF with
the reference's names (JointSettings / ObjectHandler, myfunctions.cpp:176-196, 719-787;
read_gripper_dimensions numerics, 836-953) reads back into the identical gm_model, bit
for bit, for every finger segment count and dimension variant; the loader also rejects
malformed input loudly.  A GPU test (test_mjcf_model_steps_like_the_built_one) checks that
an env built from the loaded model steps exactly like one from the built model."""
import ctypes as C
import re

import numpy as np
import pytest


def build(gm, **kw):
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return gm.ModelBlob(p)


@pytest.mark.parametrize("kw", [{}, {"n_seg": 5}, {"n_seg": 7}, {"n_seg": 6, "finger_thickness": 1.0e-3,
                                                                    "finger_width": 24e-3},
                                {"hook_angle_degrees": 90.0, "segment_inertia_scaling": 1.0, "timestep": 2e-3}])
def test_round_trip_is_bit_exact(gm, kw):
    m = build(gm, **kw)
    xml = m.to_mjcf()
    m2 = gm.ModelBlob.from_mjcf(xml)
    assert bytes(m.buf) == bytes(m2.buf)
    assert m2.to_mjcf() == xml


def test_mjcf_uses_reference_names(gm):
    xml = build(gm).to_mjcf()
    for name in ("world_to_base", "palm_prismatic_joint", "finger_1_prismatic_joint", "finger_2_revolute_joint",
                 "finger_3_segment_joint_8", "gripper_base_link", "initial pose"):
        assert f'"{name}"' in xml
    for num in ("finger_length", "finger_width", "finger_E", "fingertip_clearance", "hook_angle_degrees",
                "hook_length", "fixed_hook_segment", "fixed_first_segment"):
        assert f'<numeric name="{num}"' in xml
    assert xml.count("<pair ") == build(gm).npair
    assert len(re.findall(r"<joint name=\"[^\"]+_lock\"", xml)) == 4


def test_loader_reads_numerics_and_derives_gains(gm):
    """read_gripper_dimensions: a different finger_E in the MJCF reaches the model and the
    constants derived from it (EI, PD gains, myfunctions.cpp:273-296) change with it."""
    m = build(gm)
    xml = m.to_mjcf().replace('<numeric name="finger_E" data="193000000000"', '<numeric name="finger_E" data="100000000000"')
    assert 'data="100000000000"' in xml
    m2 = gm.ModelBlob.from_mjcf(xml)
    assert bytes(m2.buf) != bytes(m.buf)
    assert '<numeric name="finger_E" data="100000000000"/>' in m2.to_mjcf()
    # only the modulus and what derives from it differ: restoring it restores the model
    back = gm.ModelBlob.from_mjcf(m2.to_mjcf().replace('data="100000000000"', 'data="193000000000"'))
    assert bytes(back.buf) == bytes(m.buf)


@pytest.mark.parametrize("bad", ["", "<mujoco>", "<robot></robot>", "<mujoco><worldbody></worldbody></mujoco>",
                                 "<mujoco><worldbody><body name='x'><joint type='ball'/></body></worldbody></mujoco>"])
def test_loader_rejects_malformed(gm, bad):
    with pytest.raises(ValueError):
        gm.ModelBlob.from_mjcf(bad)


@pytest.mark.gpu
def test_mjcf_model_steps_like_the_built_one(gm):
    from conftest import gpu_available
    if not gpu_available():
        pytest.skip("no GPU")
    built = build(gm)
    loaded = gm.ModelBlob.from_mjcf(built.to_mjcf())
    out = []
    for model in (built, loaded):
        s = gm.canonical_settings(noise=True, seed=3)
        env = gm.BatchedGripperEnv(256, object_set="set6_synthetic", settings=s, seed=3, model_blob=model)
        env.reset()
        sc = gm.GraspScript(s, 256, seed=3)
        for k in range(50):
            env.step(sc.actions(k))
        out.append((env.observation(), env.env_states()))
        env.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
