"""Extract the nine MiniMax 13x13 maze layouts (data) from the reference.

Reads environments/gridworld/custom_mazes.py:6-163 *as text* (no import) and
writes to-ued_amd/toued/data/mazes.json: {name: [wall cell indices]} in the
order of MAZE_DESIGNS (custom_mazes.py:153-163).  Run once in the build
container; the JSON is committed so nothing reads /root/reference at run time.
"""
import json
import re
import sys
from pathlib import Path

SRC = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/environments/gridworld/custom_mazes.py")
OUT = Path(__file__).resolve().parents[1] / "to-ued_amd" / "toued" / "data" / "mazes.json"

text = SRC.read_text()
layouts = {}
for m in re.finditer(r"^(\w+) = \[(.*?)\]", text, flags=re.S | re.M):
    cells = [int(v) for v in re.findall(r"[01]", m.group(2))]
    assert len(cells) == 169, (m.group(1), len(cells))
    layouts[m.group(1)] = [i for i, v in enumerate(cells) if v == 1]
order = re.findall(r"'(\w+)': _to_wall_idxs\(\w+\)", text)
out = {name: layouts[name] for name in order}
OUT.write_text("{\n" + ",\n".join(f"  {json.dumps(k)}: {json.dumps(v)}" for k, v in out.items()) + "\n}\n")
print(f"wrote {len(out)} mazes to {OUT}")
