"""GPU: the two device PGS paths on identical contact-rich states.

The step kernel solves problems with nefc <= 32 on the replicated 16-lane-row layout
(row changes broadcast with v_mov_b64_dpp row_newbcast) and larger ones lane-per-row
with a v_readlane broadcast (csrc/gm_kernels.hip, constraints()).  Both perform the same
arithmetic operation for operation (mj_solPGS's sweep in the u-formulation), so a build
that sends every problem down the general path (lib/libgm_pgsgen.so, -DGM_PGS_GENERAL_ONLY)
must reproduce the default build's forces, accelerations and observations exactly, up to
the sign of an exact zero.  The batch is checked to contain problems of every size class
(nefc <= 16, 17..32, > 32), so each device path is held against the oracle-checked one.
"""
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

N_ENVS = 512


@pytest.fixture(scope="module")
def pair(gm):
    if not gpu_available():
        pytest.skip("no GPU")
    from gmx._lib import load_library
    from gmx.build import PGSGEN_PATH
    assert os.path.exists(PGSGEN_PATH), "run __graft_entry__.build() first (libgm_pgsgen.so missing)"
    lib_gen = load_library(PGSGEN_PATH)
    envs = []
    for lib in (None, lib_gen):
        s = gm.canonical_settings(noise=False, seed=11)
        env = gm.BatchedGripperEnv(N_ENVS, object_set="set6_synthetic", settings=s, seed=11, lib=lib)
        env.reset()
        envs.append(env)
    return envs


def test_dpp_row_pgs_matches_general_path(pair, gm):
    dflt, gen = pair
    # the scripted grasp mix drives the batch into finger / object contact, so problems
    # of every size class occur; every env-step's outputs must agree exactly
    script = gm.GraspScript(dflt.settings, N_ENVS, seed=11)
    for t in range(48):
        a = script.actions(t)
        od, rd, _, _ = dflt.step(a)
        og, rg, _, _ = gen.step(a)
        np.testing.assert_array_equal(od, og)
        np.testing.assert_array_equal(rd, rg)
    ncon, con, f, qacc = dflt.debug_substep()
    ncon_g, con_g, f_g, qacc_g = gen.debug_substep()
    np.testing.assert_array_equal(ncon, ncon_g)
    np.testing.assert_array_equal(f, f_g)
    np.testing.assert_array_equal(qacc, qacc_g)
    # size classes present: nefc = active locks (0..4) + 4 ncon
    assert (ncon <= 3).any(), np.bincount(ncon)           # nefc <= 16: one row set
    assert ((ncon >= 5) & (ncon <= 7)).any(), np.bincount(ncon)   # 17..32: two row sets
    assert (ncon >= 9).any(), np.bincount(ncon)           # > 32: general path in both builds
