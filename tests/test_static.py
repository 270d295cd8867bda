"""Static check (CPU): every global name a function of the host package reads is
defined in its module -- catches a missing import before a GPU run does."""
import builtins
import dis
import importlib
import pkgutil
import types

import pytest

MODULES = []


def _collect():
    import irc_amd
    import src

    for pkg in (irc_amd, src):
        MODULES.append(pkg.__name__)
        for m in pkgutil.walk_packages(pkg.__path__, pkg.__name__ + "."):
            MODULES.append(m.name)
    return MODULES


def _code_objects(co):
    yield co
    for c in co.co_consts:
        if isinstance(c, types.CodeType):
            yield from _code_objects(c)


@pytest.mark.parametrize("modname", _collect())
def test_no_undefined_globals(modname):
    mod = importlib.import_module(modname)
    path = getattr(mod, "__file__", None)
    if not path or not path.endswith(".py"):
        return
    src = open(path).read()
    top = compile(src, path, "exec")
    missing = set()
    for co in _code_objects(top):
        if co is top:
            continue
        for ins in dis.get_instructions(co):
            if ins.opname == "LOAD_GLOBAL":
                name = ins.argval
                if not hasattr(mod, name) and not hasattr(builtins, name):
                    missing.add((co.co_name, name))
    assert not missing, f"{modname}: undefined globals {sorted(missing)}"
