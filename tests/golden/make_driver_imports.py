"""Writes tests/golden/driver_imports.json: for every reference module that prfl_amd.dropin
replaces, the top-level names the reference module defines and every name any reference file
imports from it (absolute or relative `from ... import`), with the importing file:line.

Run here, where /root/reference exists (the reference's sources are parsed with `ast`, nothing of
them is imported or executed):  python tests/golden/make_driver_imports.py
"""
import ast
import json
import os
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "hy-video-prfl_amd"))
from prfl_amd.dropin import MODULE_MAP  # noqa: E402


def module_of(path):
    rel = os.path.relpath(path, REF)[:-3].replace(os.sep, ".")
    return rel[:-len(".__init__")] if rel.endswith(".__init__") else rel


def defined_names(path):
    names = set()
    for n in ast.parse(open(path).read()).body:
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            names.add(n.name)
        elif isinstance(n, (ast.Assign, ast.AnnAssign)):
            for t in (n.targets if isinstance(n, ast.Assign) else [n.target]):
                if isinstance(t, ast.Name):
                    names.add(t.id)
    return sorted(x for x in names if not x.startswith("_") or x == "__all__")


def imports(path):
    """Yield (absolute module, name, line) for every `from X import name` in the file."""
    me = module_of(path)
    pkg = me if path.endswith("__init__.py") else me.rpartition(".")[0]
    for n in ast.walk(ast.parse(open(path).read())):
        if not isinstance(n, ast.ImportFrom):
            continue
        if n.level:
            base = pkg.split(".")
            base = base[:len(base) - (n.level - 1)]
            mod = ".".join(base + ([n.module] if n.module else []))
        else:
            mod = n.module or ""
        for a in n.names:
            yield mod, a.name, n.lineno


def main():
    out = {}
    for ref_mod in MODULE_MAP:
        out[ref_mod] = {"defined": defined_names(os.path.join(REF, *ref_mod.split(".")) + ".py"),
                        "imported": {}}
    for root, _, files in os.walk(REF):
        for f in files:
            if not f.endswith(".py"):
                continue
            p = os.path.join(root, f)
            for mod, name, line in imports(p):
                if mod in out:
                    out[mod]["imported"].setdefault(name, []).append(
                        f"{os.path.relpath(p, REF)}:{line}")
    for v in out.values():
        v["imported"] = {k: sorted(s) for k, s in sorted(v["imported"].items())}
    with open(os.path.join(HERE, "driver_imports.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({k: len(v["imported"]) for k, v in out.items()}))


if __name__ == "__main__":
    main()
