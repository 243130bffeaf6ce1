"""ctypes binding of libvcg_hip.so.

The argument types are derived from the C prototypes in `include/vcg_hip.h` (the single source
of truth for the ABI), so the Python side can never drift from the header. The library must be
loaded after torch so that it shares torch's HIP runtime (both carry SONAME libamdhip64.so.7).
There is no fallback: if the library is missing or fails to load, every op raises.
"""
import ctypes
import os
import re
import threading

import torch  # noqa: F401  (must be imported first: provides the HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VCG_LIB_PATH") or os.path.join(_HERE, "libvcg_hip.so")  # override: A/B builds


def _find_header():
    cands = [
        os.path.join(_HERE, "vcg_hip.h"),
        os.path.join(_HERE, "..", "..", "include", "vcg_hip.h"),
    ]
    for c in cands:
        if os.path.exists(c):
            return os.path.abspath(c)
    raise RuntimeError("vcg_hip.h not found next to the package or under include/")


HEADER_PATH = _find_header()

_CTYPE = {
    "int": ctypes.c_int,
    "long long": ctypes.c_longlong,
    "unsigned long long": ctypes.c_ulonglong,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "hipStream_t": ctypes.c_void_p,
    "void": None,
}


def _parse_type(t):
    t = t.strip()
    t = re.sub(r"\bconst\b", "", t).strip()
    if "*" in t:
        base = t.replace("*", "").strip()
        if base == "char":
            return ctypes.c_char_p
        return ctypes.c_void_p
    if t not in _CTYPE:
        raise RuntimeError(f"unhandled C type '{t}' in {HEADER_PATH}")
    return _CTYPE[t]


def parse_header(path=HEADER_PATH):
    """Return {name: (restype, [argtypes], [argnames])} for every VCG_API prototype."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"VCG_API\s+([\w\s\*]+?)\s*\b(vcg_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        argtypes, argnames = [], []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                mm = re.match(r"(.*?)(\w+)$", a)
                typ, nm = mm.group(1), mm.group(2)
                argtypes.append(_parse_type(typ))
                argnames.append(nm)
        protos[name] = (_parse_type(ret), argtypes, argnames)
    return protos


PROTOS = parse_header()

_lib = None
_lock = threading.Lock()


class VcgError(RuntimeError):
    pass


def lib():
    """Load libvcg_hip.so (once). Raises loudly if it is absent or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise VcgError(
                f"libvcg_hip.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, argt, _) in PROTOS.items():
            fn = getattr(handle, name)  # AttributeError = header/library mismatch: fail loudly
            fn.restype = res
            fn.argtypes = argt
        _lib = handle
    return _lib


def last_error():
    return lib().vcg_last_error().decode()


def call(name, *args):
    """Invoke a status-returning entry point; raise VcgError with the library message on failure."""
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise VcgError(f"{name} failed ({rc}): {last_error()}")
    return rc


def query(name, *args):
    """Invoke a size-query entry point (returns a value, not a status)."""
    return getattr(lib(), name)(*args)
