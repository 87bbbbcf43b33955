"""Every global name the package's functions load is defined in their module or a builtin (a
pruned knob that left a reader behind fails here on the CPU instead of in a GPU run)."""
import builtins
import dis
import importlib
import os
import pkgutil
import types

import quantizers_amd


def _functions(mod):
    for v in list(vars(mod).values()):
        if isinstance(v, types.FunctionType):
            yield v
        elif isinstance(v, type) and v.__module__ == mod.__name__:
            for f in vars(v).values():
                if isinstance(f, (staticmethod, classmethod)):
                    f = f.__func__
                elif isinstance(f, property):
                    f = f.fget
                if isinstance(f, types.FunctionType):
                    yield f


def _code_objects(co):
    yield co
    for c in co.co_consts:
        if isinstance(c, types.CodeType):
            yield from _code_objects(c)


def test_no_undefined_globals():
    missing = []
    names = [i.name for i in pkgutil.walk_packages(quantizers_amd.__path__, "quantizers_amd.")
             if not i.name.endswith("libquantizers_amd")] + ["bench", "__graft_entry__"]
    for name in names:
        mod = importlib.import_module(name)
        src = os.path.realpath(mod.__file__)
        for f in _functions(mod):
            if os.path.realpath(f.__code__.co_filename) != src:
                continue  # a decorator's wrapper from another module
            for co in _code_objects(f.__code__):
                for ins in dis.get_instructions(co):
                    if ins.opname == "LOAD_GLOBAL" and ins.argval not in vars(mod) and not hasattr(builtins, ins.argval):
                        missing.append(f"{name}.{co.co_name}: {ins.argval}")
    assert not missing, missing
