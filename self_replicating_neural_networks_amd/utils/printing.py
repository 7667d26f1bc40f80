"""Silence-able printing mixin (reference code/util.py:1-39, ``PrintingObject``)."""
from __future__ import annotations

import contextlib


class PrintingObject:
    """Objects that print debug output only when not silent (default: silent)."""

    class SilenceSignal:
        """Context manager that temporarily sets an object's silence flag."""

        def __init__(self, obj, value):
            self.obj = obj
            self.new_silent = value
            self.old_silent = None

        def __enter__(self):
            self.old_silent = self.obj.get_silence()
            self.obj.set_silence(self.new_silent)
            return self.obj

        def __exit__(self, exc_type, exc, tb):
            self.obj.set_silence(self.old_silent)
            return False

    def __init__(self):
        self.silent = True

    def is_silent(self) -> bool:
        return self.silent

    def get_silence(self) -> bool:
        return self.is_silent()

    def set_silence(self, value: bool = True):
        self.silent = value
        return self

    def unset_silence(self):
        self.silent = False
        return self

    def with_silence(self, value: bool = True):
        return self.set_silence(value)

    def silence(self, value: bool = True):
        return self.__class__.SilenceSignal(self, value)

    def _print(self, *args, **kwargs):
        if not self.silent:
            print(*args, **kwargs)


@contextlib.contextmanager
def silenced(*objs):
    olds = [o.get_silence() for o in objs]
    for o in objs:
        o.set_silence(True)
    try:
        yield
    finally:
        for o, v in zip(objs, olds):
            o.set_silence(v)
