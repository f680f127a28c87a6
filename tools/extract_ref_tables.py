"""Extract the reference's data tables (data, not code) into tests/golden/ref_tables.json.

Reads, as text and through Python's `ast` module -- never importing or executing them:
  * environments/gridworld/configs.py:148-707  ENV_MODE_PARAMS / ENV_MODE_KWARGS / ENV_MODE_EPISODE_LEN /
    ENV_MODE_LIFETIME / ENV_MODE_LIFETIME_MAX / MODE_AGENT_HYPERS;
  * environments/gridworld/custom_mazes.py:6-163  the maze layouts (MAZE_DESIGNS, wall cell indices);
  * experiments/parse_args.py:5-204  every add_argument's flags, dest, type, action and default.

The table expressions are folded by a small whitelisted evaluator over the AST: literals, list/tuple/dict displays
(incl. ``**`` merges and comprehensions over known names), ``list * int``, integer arithmetic, subscripts of known
tables, ``jnp.array([...])``, ``jnp.argwhere`` over ``jnp.arange`` / comparisons / ``logical_*`` / ``isin`` (numpy),
``lambda _: X`` and ``partial(fn, ...)``.  A ``partial`` distribution is written as the spec tuple the oracle's
tables use (oracle/modes.py docstring): ("log_uniform_int", lo, hi), ("log_uniform", n, lo, hi),
("uniform", n, lo, hi), ("uniform_first_pos", n, lo, hi), ("choice_arange", lo, hi), ("wall_idxs", n_walls, max_grid);
a constant as ("const", v).  Anything else raises, so a change of the reference's tables cannot pass unnoticed.

Run once in the build container (``python tools/extract_ref_tables.py``); the JSON is committed and
tests/test_ref_tables.py compares oracle/modes.py, toued/modes.py and toued/parse_args.py against it.  Nothing reads
/root/reference at test or run time.
"""
from __future__ import annotations

import ast
import json
import re
import sys
from pathlib import Path

import numpy as np

REF = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden" / "ref_tables.json"

CONST_FIELDS = ("max_steps_in_episode", "obj_rewards", "obj_p_terminate", "obj_p_respawn", "n_objs", "grid_size",
                "wall_idxs")


class Partial:
    def __init__(self, fn, kw):
        self.fn, self.kw = fn, kw


class Lambda:
    def __init__(self, value):
        self.value = value


def _dotted(node):
    if isinstance(node, ast.Name):
        return node.id
    if isinstance(node, ast.Attribute):
        return _dotted(node.value) + "." + node.attr
    raise ValueError(f"unsupported callee {ast.dump(node)}")


class Folder:
    """Folds the whitelisted expression forms; ``env`` holds the module-level names evaluated so far."""

    def __init__(self, env):
        self.env = env

    def ev(self, n, local=None):
        local = local or {}
        if isinstance(n, ast.Constant):
            return n.value
        if isinstance(n, (ast.List, ast.Tuple)):
            return [self.ev(e, local) for e in n.elts]
        if isinstance(n, ast.Name):
            if n.id in local:
                return local[n.id]
            if n.id in self.env:
                return self.env[n.id]
            raise KeyError(n.id)
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.USub):
            return -self.ev(n.operand, local)
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.Not):
            return np.logical_not(self.ev(n.operand, local))
        if isinstance(n, ast.BinOp):
            a, b = self.ev(n.left, local), self.ev(n.right, local)
            op = type(n.op)
            if op is ast.Mult:
                if isinstance(a, list) and isinstance(b, int):
                    return a * b
                if isinstance(b, list) and isinstance(a, int):
                    return a * b
                return a * b
            if op is ast.FloorDiv:
                return a // b
            if op is ast.Mod:
                return a % b
            if op is ast.Add:
                return a + b
            if op is ast.Sub:
                return a - b
            if op is ast.Pow:
                return a ** b
            raise ValueError(f"unsupported operator {op.__name__}")
        if isinstance(n, ast.Compare) and len(n.ops) == 1 and isinstance(n.ops[0], ast.Eq):
            return self.ev(n.left, local) == self.ev(n.comparators[0], local)
        if isinstance(n, ast.Subscript):
            return self.ev(n.value, local)[self.ev(n.slice, local)]
        if isinstance(n, ast.Dict):
            out = {}
            for k, v in zip(n.keys, n.values):
                if k is None:
                    out.update(self.ev(v, local))
                else:
                    out[self.ev(k, local)] = self.ev(v, local)
            return out
        if isinstance(n, ast.DictComp):
            (gen,) = n.generators
            out = {}
            for item in self.ev(gen.iter, local):
                loc = dict(local, **{gen.target.id: item})
                out[self.ev(n.key, loc)] = self.ev(n.value, loc)
            return out
        if isinstance(n, ast.Lambda):
            return Lambda(self.ev(n.body, local))
        if isinstance(n, ast.Attribute) and _dotted(n) in ("jnp.int32", "jnp.float32"):
            return _dotted(n)       # a dtype argument
        if isinstance(n, ast.Call):
            return self.call(n, local)
        raise ValueError(f"unsupported expression {ast.dump(n)[:120]}")

    def call(self, n, local):
        fn = _dotted(n.func)
        kw = {k.arg: self.ev(k.value, local) for k in n.keywords}
        if fn == "partial":         # the distribution by name; its keyword arguments folded
            assert len(n.args) == 1
            return Partial(_dotted(n.args[0]), kw)
        args = [self.ev(a, local) for a in n.args]
        if fn == "jnp.array":
            return [x for x in np.asarray(args[0]).reshape(-1).tolist()]
        if fn == "jnp.arange":
            return np.arange(*args)
        if fn == "jnp.logical_and":
            return np.logical_and(*args)
        if fn == "jnp.logical_or":
            return np.logical_or(*args)
        if fn == "jnp.logical_not":
            return np.logical_not(*args)
        if fn == "jnp.isin":
            return np.isin(np.asarray(args[0]), np.asarray(args[1]))
        if fn == "jnp.argwhere":
            return [int(i) for i in np.argwhere(np.asarray(args[0])).reshape(-1)]
        if fn == "tuple":
            return list(args[0])
        if fn == "int":
            return int(args[0])
        if fn in self.env and isinstance(self.env[fn], ast.FunctionDef):
            return self.run_function(self.env[fn], args)
        raise ValueError(f"unsupported call {fn}")

    def run_function(self, fdef, args):
        """A function body of assignments (to names and to subscripts) and one return, e.g. get_maze_params."""
        loc = {a.arg: v for a, v in zip(fdef.args.args, args)}
        for st in fdef.body:
            if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Name):
                loc[st.targets[0].id] = self.ev(st.value, loc)
            elif isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Subscript):
                t = st.targets[0]
                self.ev(t.value, loc)[self.ev(t.slice, loc)] = self.ev(st.value, loc)
            elif isinstance(st, ast.Return):
                return self.ev(st.value, loc)
            elif isinstance(st, ast.Expr) and isinstance(st.value, ast.Constant):
                continue
            else:
                raise ValueError(f"unsupported statement in {fdef.name}: {ast.dump(st)[:120]}")
        raise ValueError(f"{fdef.name} has no return")


def spec(v, field=None):
    """A folded value as the oracle's spec tuple (a list in JSON)."""
    if isinstance(v, Partial):
        kw = v.kw
        if v.fn == "log_uniform_int":
            assert tuple(kw["shape"]) == (), kw
            return ["log_uniform_int", kw["minval"], kw["maxval"]]
        if v.fn == "log_uniform":
            (n,) = kw["shape"]
            return ["log_uniform", n, kw["minval"], kw["maxval"]]
        if v.fn == "random.uniform":
            (n,) = kw["shape"]
            return ["uniform", n, kw["minval"], kw["maxval"]]
        if v.fn == "uniform_first_pos":
            return ["uniform_first_pos", kw["n"], kw["minval"], kw["maxval"]]
        if v.fn == "random.choice":
            a = np.asarray(kw["a"])
            assert np.array_equal(a, np.arange(a[0], a[-1] + 1)), a
            return ["choice_arange", int(a[0]), int(a[-1]) + 1]
        if v.fn == "uniform_wall_idxs":
            return ["wall_idxs", kw["n_walls"], kw["max_grid_size"]]
        raise ValueError(f"unknown distribution {v.fn}")
    if isinstance(v, Lambda):
        return ["const", v.value]
    return ["const", v]


def mazes(text):
    """custom_mazes.py: the 13x13 0/1 layouts and MAZE_DESIGNS' order (same reading as tools/extract_mazes.py)."""
    layouts = {}
    for m in re.finditer(r"^(\w+) = \[(.*?)\]", text, flags=re.S | re.M):
        cells = [int(v) for v in re.findall(r"[01]", m.group(2))]
        assert len(cells) == 169, (m.group(1), len(cells))
        layouts[m.group(1)] = [i for i, v in enumerate(cells) if v == 1]
    order = re.findall(r"'(\w+)': _to_wall_idxs\(\w+\)", text)
    return {name: layouts[name] for name in order}


def configs_tables(text, maze_designs):
    tree = ast.parse(text)
    env = {"MAZE_DESIGNS": maze_designs}
    fold = Folder(env)
    for st in tree.body:
        if isinstance(st, ast.FunctionDef):
            env[st.name] = st
        elif isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Name):
            name = st.targets[0].id
            try:
                env[name] = fold.ev(st.value)
            except (KeyError, ValueError):
                if name in ("ENV_MODE_PARAMS", "ENV_MODE_KWARGS", "ENV_MODE_EPISODE_LEN", "ENV_MODE_LIFETIME",
                            "ENV_MODE_LIFETIME_MAX", "MODE_AGENT_HYPERS") or name.startswith("_"):
                    raise
        elif isinstance(st, ast.Expr) and isinstance(st.value, ast.Call) and \
                _dotted(st.value.func) == "ENV_MODE_LIFETIME_MAX.update":
            # configs.py:644-650: the deterministic lifetimes are the lambdas' values, added where not already set
            for mode, f in env["ENV_MODE_LIFETIME"].items():
                if mode not in env["ENV_MODE_LIFETIME_MAX"]:
                    assert isinstance(f, Lambda), mode
                    env["ENV_MODE_LIFETIME_MAX"][mode] = f.value
    params = {}
    for mode, p in env["ENV_MODE_PARAMS"].items():
        if p.get("manual"):
            params[mode] = {"manual": True, "modes": list(p["modes"])}
            continue
        q = {"manual": False, "obj_ids": list(p["obj_ids"]), "tabular": p["tabular"], "auto_collect": p["auto_collect"]}
        for f in CONST_FIELDS:
            q[f] = spec(p[f], f)
        params[mode] = q
    hypers = {m: {k: (list(v) if isinstance(v, (list, tuple)) else v) for k, v in h.items()}
              for m, h in env["MODE_AGENT_HYPERS"].items()}
    return {
        "ENV_MODE_PARAMS": params,
        "ENV_MODE_KWARGS": env["ENV_MODE_KWARGS"],
        "ENV_MODE_EPISODE_LEN": env["ENV_MODE_EPISODE_LEN"],
        "ENV_MODE_LIFETIME": {m: spec(v) for m, v in env["ENV_MODE_LIFETIME"].items()},
        "ENV_MODE_LIFETIME_MAX": env["ENV_MODE_LIFETIME_MAX"],
        "MODE_AGENT_HYPERS": hypers,
    }


def parse_args_defaults(text):
    """Every parser.add_argument(...) of parse_args.py: {dest: {flags, type, action, default}}."""
    tree = ast.parse(text)
    fold = Folder({})
    out = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr == "add_argument":
            flags = [a.value for a in node.args]
            kw = {k.arg: k.value for k in node.keywords}
            long = next(f for f in flags if f.startswith("--"))
            dest = kw["dest"].value if "dest" in kw else long[2:].replace("-", "_")
            action = kw["action"].value if "action" in kw else None
            typ = kw["type"].id if "type" in kw else None
            if "default" in kw:
                default = fold.ev(kw["default"])
            else:
                default = False if action == "store_true" else None
            out[dest] = {"flags": flags, "type": typ, "action": action, "default": default}
    return out


def main():
    md = mazes((REF / "environments/gridworld/custom_mazes.py").read_text())
    tables = configs_tables((REF / "environments/gridworld/configs.py").read_text(), md)
    tables["MAZE_DESIGNS"] = md
    tables["parse_args"] = parse_args_defaults((REF / "experiments/parse_args.py").read_text())
    tables["_source"] = {"configs": "environments/gridworld/configs.py:129-707",
                         "mazes": "environments/gridworld/custom_mazes.py:6-163",
                         "parse_args": "experiments/parse_args.py:5-204",
                         "generator": "tools/extract_ref_tables.py"}
    OUT.write_text(json.dumps(tables, indent=1, sort_keys=True) + "\n")
    print(f"wrote {OUT}: {len(tables['ENV_MODE_PARAMS'])} modes, {len(tables['parse_args'])} flags")


if __name__ == "__main__":
    main()
