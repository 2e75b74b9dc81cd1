"""Observation samplers and the cartesian contact stream, device vs oracle on grasp
states.  MjClass::configure_settings picks one of seven window samplers for the sensor
streams and one for the state streams (mjclass.cpp:144-211; raw, change, average, median,
sign, scaled_change, scaled_change_sq, mjclass.h:278-453), and the optional
cartesian_contacts_XYZ stream samples the per-finger contact positions
(mjclass.cpp:1889-1959).  The canonical config exercises one pair; here every mode runs
on both stream kinds, with the cartesian stream on, through the same step comparison as
tests/test_grasp_parity.py (observations, done flags, event rows, reward)."""
import pytest

from test_grasp_parity import compare_step, rollout, ol  # noqa: F401  (ol: fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sensor_mode", range(7))
def test_sampler_modes_match_oracle(gm, ol, sensor_mode):
    state_mode = (sensor_mode + 3) % 7

    def modes(s):
        s.sensor_sample_mode = sensor_mode
        s.state_sample_mode = state_mode
        s.cartesian_contacts_XYZ.in_use = 1

    env, snaps = rollout(gm, 256, "set6_synthetic", 500 + sensor_mode, steps=45, snaps=(20, 44), tweak=modes)
    base = gm.ConfigBlob(gm.canonical_settings(seed=1), env.model).n_obs
    assert env.cfg.n_obs > base, "the cartesian stream did not add observations"
    rep = [compare_step(gm, ol, env, sn) for sn in snaps]
    print(f"sensor mode {sensor_mode} / state mode {state_mode}: {rep}")
    env.close()
