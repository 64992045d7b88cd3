"""Shared loader of the tree's libecorr.so and the AB_ALT_LIB lab libraries (name=path,...)."""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    from eraft_amd import _lib
    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SYMBOLS.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            continue
        fn.restype = res
        fn.argtypes = args
    return L


def load_libs():
    from eraft_amd import _lib
    libs = {"tree": load(_lib.LIB_PATH)}
    for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
        name, _, path = item.rpartition("=")
        libs[name or f"alt{k}"] = load(os.path.join(ROOT, path))
    return libs
