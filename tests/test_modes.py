"""The product's mode tables (toued/modes.py) equal the oracle's restatement."""
import numpy as np

from oracle import modes as om


def test_tables_identical():
    from toued import modes as pm
    for name in ("ENV_MODE_PARAMS", "ENV_MODE_KWARGS", "ENV_MODE_EPISODE_LEN", "ENV_MODE_LIFETIME",
                 "ENV_MODE_LIFETIME_MAX", "MODE_AGENT_HYPERS", "MAZE_DESIGNS"):
        assert getattr(om, name) == getattr(pm, name), name


def test_obs_dims_match_survey():
    from oracle.levels import env_spec
    assert env_spec("tabular").obs_dim == 5409
    assert env_spec("all_shortlife").obs_dim == 3201
    assert env_spec("mazes").obs_dim == 1353
    assert env_spec("dense").obs_dim == 1937


def test_mode_program_encodes():
    from toued import modes as pm
    for mode in pm.ENV_MODE_PARAMS:
        prog = pm.mode_program(mode)
        assert prog.dtype == np.int32 and prog.shape == (pm.PROGRAM_WORDS,)
