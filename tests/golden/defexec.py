"""Guarded execution of the reference's Python definition code — fixture GENERATION only.

The golden generators (make_golden.py, make_schema_golden.py) pin the oracle against the outputs of
the reference's own runnable definitions (a `reference` code string inside each definition JSON).
That checkout is untrusted public content, so its code is never run implicitly:

  * the generators refuse to run without the explicit opt-in flag EXEC_FLAG;
  * before execution the code is parsed and checked against an allowlist: imports only of
    ALLOWED_MODULES, no dunder attribute access, no call of a name in FORBIDDEN_NAMES;
  * it executes with a reduced builtins table whose __import__ admits only ALLOWED_MODULES.

This is a tripwire for code that does more than arithmetic on tensors, not a sandbox against a
determined attacker. The committed fixtures hold inputs and outputs only (no reference text), and
tests never call this module: they read the fixtures.
"""
from __future__ import annotations

import ast
import builtins
import hashlib
import json

EXEC_FLAG = "--exec-reference-definitions"
ALLOWED_MODULES = {"torch", "struct", "math", "numpy"}
FORBIDDEN_NAMES = {"exec", "eval", "compile", "open", "__import__", "globals", "locals", "vars", "getattr",
                   "setattr", "delattr", "input", "breakpoint", "memoryview", "help", "exit", "quit"}
SAFE_BUILTINS = ["abs", "all", "any", "bool", "bytes", "bytearray", "dict", "enumerate", "float", "int",
                 "isinstance", "len", "list", "max", "min", "pow", "range", "reversed", "round", "slice",
                 "sorted", "sum", "tuple", "zip", "ValueError", "AssertionError", "TypeError", "IndexError",
                 "Exception", "True", "False", "None"]


class DefinitionRejected(RuntimeError):
    pass


def check_source(src: str, origin: str) -> None:
    tree = ast.parse(src, origin)
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            mods = [a.name.split(".")[0] for a in node.names]
        elif isinstance(node, ast.ImportFrom):
            mods = [(node.module or "").split(".")[0]]
        else:
            mods = []
        for m in mods:
            if m not in ALLOWED_MODULES:
                raise DefinitionRejected(f"{origin}: import of {m!r} is not allowed")
        if isinstance(node, ast.Attribute) and node.attr.startswith("__"):
            raise DefinitionRejected(f"{origin}: dunder attribute {node.attr!r}")
        if isinstance(node, ast.Name) and node.id in FORBIDDEN_NAMES:
            raise DefinitionRejected(f"{origin}: use of {node.id!r}")


def _guarded_import(name, globals=None, locals=None, fromlist=(), level=0):
    if level != 0 or name.split(".")[0] not in ALLOWED_MODULES:
        raise DefinitionRejected(f"import of {name!r} is not allowed")
    return builtins.__import__(name, globals, locals, fromlist, level)


def load_definition_fn(json_path: str, fn: str = "run"):
    """(spec, callable, sha256 of the code string) for one definition JSON, after the checks above."""
    with open(json_path) as f:
        spec = json.load(f)
    src = spec["reference"]
    check_source(src, json_path)
    table = {n: getattr(builtins, n) for n in SAFE_BUILTINS if hasattr(builtins, n)}
    table["__import__"] = _guarded_import
    ns: dict = {"__builtins__": table, "__name__": "definition"}
    exec(compile(src, json_path, "exec"), ns)
    return spec, ns[fn], hashlib.sha256(src.encode()).hexdigest()


def require_opt_in(argv_flag: bool, script: str) -> None:
    if not argv_flag:
        raise SystemExit(f"{script}: refusing to execute the reference's definition code without {EXEC_FLAG} "
                         "(the committed fixtures are already generated; see tests/golden/defexec.py)")
