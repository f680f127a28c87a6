"""The oracle's and the product's data tables equal the reference's own (pinned data, not a restatement).

tests/golden/ref_tables.json is extracted from the reference's source text by tools/extract_ref_tables.py (AST folding,
no import): environments/gridworld/configs.py:129-707 (mode params, kwargs, episode lengths, lifetimes, agent hypers),
custom_mazes.py:6-163 (maze layouts) and experiments/parse_args.py:5-204 (every flag's dest, type, action, default).
"""
import argparse
import json
from pathlib import Path

import pytest

from oracle import modes as om

REF = json.loads((Path(__file__).parent / "golden" / "ref_tables.json").read_text())


def _norm(v):
    if isinstance(v, (list, tuple)):
        return [_norm(x) for x in v]
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    return v


def _modules():
    from toued import modes as pm
    return [("oracle", om), ("product", pm)]


@pytest.mark.parametrize("which", ["oracle", "product"])
def test_mode_params_pinned(which):
    mod = dict(_modules())[which]
    ref = REF["ENV_MODE_PARAMS"]
    assert sorted(mod.ENV_MODE_PARAMS) == sorted(ref)
    for mode, rp in ref.items():
        got = _norm(mod.ENV_MODE_PARAMS[mode])
        if not rp["manual"]:
            # the restatement has no auto_collect field: every reference mode sets it True, which is what the
            # device step and the level records assume (gridworld.py:96-99; level word L_AUTOC)
            assert rp["auto_collect"] is True, mode
            rp = {k: v for k, v in rp.items() if k != "auto_collect"}
        assert got == rp, mode


@pytest.mark.parametrize("which", ["oracle", "product"])
@pytest.mark.parametrize("table", ["ENV_MODE_KWARGS", "ENV_MODE_EPISODE_LEN", "ENV_MODE_LIFETIME",
                                   "ENV_MODE_LIFETIME_MAX", "MODE_AGENT_HYPERS", "MAZE_DESIGNS"])
def test_tables_pinned(which, table):
    mod = dict(_modules())[which]
    assert _norm(getattr(mod, table)) == REF[table], table


def test_parse_args_defaults_pinned():
    """Every reference flag exists here with the same option strings, dest, type, action and default."""
    from toued.parse_args import build_parser
    p = build_parser()
    acts = {a.dest: a for a in p._actions if not isinstance(a, argparse._HelpAction)}
    types = {int: "int", float: "float", str: "str", None: None}
    for dest, ref in REF["parse_args"].items():
        assert dest in acts, dest
        a = acts[dest]
        assert list(a.option_strings) == ref["flags"], dest
        assert a.default == ref["default"], (dest, a.default, ref["default"])
        assert types[a.type] == ref["type"], dest
        if ref["action"] == "store_true":
            assert isinstance(a, argparse._StoreTrueAction), dest
        else:
            assert isinstance(a, argparse._StoreAction), dest
    # the flags added here (reference-compatible extensions) are documented in toued/parse_args.py
    extra = sorted(set(acts) - set(REF["parse_args"]))
    assert all(p.get_default(d) is not None or d == "checkpoint_dir" for d in extra), extra
