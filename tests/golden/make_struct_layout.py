"""Writes tests/golden/struct_layout.json: the ctypes layout (size, and per
field its name, offset, size and ctypes type name) of every Structure in the
reference's structures.py (build container only).  Data only: no reference
source is stored.

The reference file is never executed: `parse_reference` reads it with `ast`
and rebuilds each Structure from the literal `_fields_` lists, resolving only
ctypes type names, `POINTER(...)`, module-level aliases (`Pixel = c_double`)
and Structures defined earlier in the same file.  Anything else is an error.

    python tests/golden/make_struct_layout.py"""
import ast
import ctypes
import json
import os

REF = "/root/reference/structures.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "struct_layout.json")


def layout(mod):
    out = {}
    for name in sorted(dir(mod)):
        o = getattr(mod, name)
        if isinstance(o, type) and issubclass(o, ctypes.Structure) and o is not ctypes.Structure:
            out[name] = {"size": ctypes.sizeof(o),
                         "fields": [[f[0], getattr(o, f[0]).offset, getattr(o, f[0]).size, f[1].__name__]
                                    for f in o._fields_]}
    return out


class _Namespace:
    pass


def _resolve(node, env):
    """A ctypes type from a type expression of the reference file."""
    if isinstance(node, ast.Name):
        if node.id in env:
            return env[node.id]
        if node.id.startswith("c_") and hasattr(ctypes, node.id):
            return getattr(ctypes, node.id)
    elif isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) and node.value.id == "ctypes":
        if node.attr.startswith("c_") and hasattr(ctypes, node.attr):
            return getattr(ctypes, node.attr)
    elif isinstance(node, ast.Call) and len(node.args) == 1 and not node.keywords:
        f = node.func
        is_ptr = (isinstance(f, ast.Name) and f.id == "POINTER") or (
            isinstance(f, ast.Attribute) and f.attr == "POINTER"
            and isinstance(f.value, ast.Name) and f.value.id == "ctypes")
        if is_ptr:
            return ctypes.POINTER(_resolve(node.args[0], env))
    raise ValueError(f"unsupported type expression at line {getattr(node, 'lineno', '?')}")


def parse_reference(path=REF):
    """The reference's Structures, rebuilt from its `_fields_` literals (no code run)."""
    tree = ast.parse(open(path).read(), filename=path)
    env, ns = {}, _Namespace()
    for stmt in tree.body:
        if isinstance(stmt, ast.Assign) and len(stmt.targets) == 1 and isinstance(stmt.targets[0], ast.Name):
            try:                                            # module-level alias, e.g. Pixel = c_double
                env[stmt.targets[0].id] = _resolve(stmt.value, env)
            except ValueError:
                pass
        elif isinstance(stmt, ast.ClassDef):
            fields = None
            for s in stmt.body:
                if (isinstance(s, ast.Assign) and len(s.targets) == 1 and isinstance(s.targets[0], ast.Name)
                        and s.targets[0].id == "_fields_"):
                    fields = [(ast.literal_eval(e.elts[0]), _resolve(e.elts[1], env)) for e in s.value.elts]
            if fields is None:
                continue
            cls = type(stmt.name, (ctypes.Structure,), {"_fields_": fields})
            env[stmt.name] = cls
            setattr(ns, stmt.name, cls)
    return ns


if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump(layout(parse_reference()), f, indent=1, sort_keys=True)
    print("wrote", OUT)
