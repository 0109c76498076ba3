"""Writes tests/golden/struct_layout.json: the ctypes layout (size, and per
field its name, offset, size and ctypes type name) of every Structure in the
reference's structures.py, loaded by importlib from /root/reference (build
container only).  Data only: no reference source is stored.

    python tests/golden/make_struct_layout.py"""
import ctypes
import importlib.util
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


def load_reference():
    spec = importlib.util.spec_from_file_location("ref_structures", REF)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump(layout(load_reference()), f, indent=1, sort_keys=True)
    print("wrote", OUT)
