"""Derive the traversal-order tables of the reference shader into a test fixture.

The authoritative tables are data in /root/reference/shaders/octree_fragment_shader.glsl:352-447:
a chain of `if (comparitor == vec3(...) || ...)` clauses, each followed by eight
`traversalOrder[i] = v;` assignments.  This script parses that chain (no hand-typing) and
writes tests/golden/traversal_orders.json: per clause the sign vectors it tests, the order it
assigns and the shader lines it came from, plus the SHA-256 of the shader file.  The CPU suite
checks the oracle's table and the kernel's closed form (order[r] = perm(r) ^ m) against it
(tests/test_math.py).  Run in the build container (the reference is not on the GPU box):
    python tools/extract_orders.py [shader path] [out json]
"""
import hashlib
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SHADER = Path("/root/reference/shaders/octree_fragment_shader.glsl")
OUT = ROOT / "tests" / "golden" / "traversal_orders.json"

VEC = re.compile(r"comparitor\s*==\s*vec3\(\s*([-+0-9.]+)\s*,\s*([-+0-9.]+)\s*,\s*([-+0-9.]+)\s*\)")
ASSIGN = re.compile(r"traversalOrder\[(\d)\]\s*=\s*(\d)\s*;")
COMMENT = re.compile(r"//\s*(.+?)\s*$")


def extract(text: str):
    lines = text.splitlines()
    clauses = []
    cur = None
    in_cond = False
    for no, line in enumerate(lines, 1):
        if "comparitor ==" in line and ("if (" in line or in_cond):
            if "if (" in line:
                cur = {"sign_vectors": [], "order": [None] * 8, "name": "", "lines": [no, no]}
                clauses.append(cur)
            in_cond = not line.rstrip().endswith("{")
            for m in VEC.finditer(line):
                cur["sign_vectors"].append([int(float(c)) for c in m.groups()])
            cur["lines"][1] = no
            continue
        if cur is None:
            continue
        m = ASSIGN.search(line)
        if m:
            cur["order"][int(m.group(1))] = int(m.group(2))
            cur["lines"][1] = no
            continue
        c = COMMENT.search(line)
        if c and not cur["name"] and all(v is None for v in cur["order"]):
            cur["name"] = c.group(1)
        if "Process children" in line:
            break
    for c in clauses:
        if any(v is None for v in c["order"]) or sorted(c["order"]) != list(range(8)):
            raise SystemExit(f"clause at lines {c['lines']} is not a permutation: {c['order']}")
    return clauses


def main():
    src = Path(sys.argv[1]) if len(sys.argv) > 1 else SHADER
    out = Path(sys.argv[2]) if len(sys.argv) > 2 else OUT
    data = src.read_bytes()
    clauses = extract(data.decode())
    vecs = [tuple(v) for c in clauses for v in c["sign_vectors"]]
    if len(vecs) != 26 or len(set(vecs)) != 26 or (0, 0, 0) in vecs:
        raise SystemExit(f"expected the 26 non-zero sign vectors once each, got {len(vecs)}")
    rec = {"source": "shaders/octree_fragment_shader.glsl (Tiago27Cruz/OctreeRayTracer)",
           "source_sha256": hashlib.sha256(data).hexdigest(),
           "generator": "tools/extract_orders.py",
           "clauses": clauses}
    out.write_text(json.dumps(rec, indent=1) + "\n")
    print(f"{len(clauses)} clauses, {len(vecs)} sign vectors -> {out}")


if __name__ == "__main__":
    main()
