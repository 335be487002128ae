"""Read the reference's designed height maps WITHOUT unpickling them.

The reference's DOE ``.save()`` (Components/QuantizedDOE.py:253-267) writes
``np.save(path, {'thickness': float32 [H, W], 'dxy': array})``: a 0-d numpy OBJECT array, i.e. a
pickle stream behind the .npy header.  ``np.load(allow_pickle=False)`` refuses it, and this build
never runs a pickle loader (pickle / numpy allow_pickle / a restricted Unpickler) on files that
ship with the reference.

This module is a data parser instead: ``pickletools.genops`` tokenises the stream (it constructs
no object and resolves no global), and a ten-opcode literal evaluator rebuilds exactly the
structure ``.save()`` writes -- a dict of str -> ndarray -- from the raw array bytes the stream
carries.  The only globals the stream may name are numpy's array reconstructor, ``numpy.ndarray``
and ``numpy.dtype``; they are matched by name to this module's own constructors
(``np.frombuffer`` on the carried bytes), never imported from the file.  Anything else -- another
global, an opcode outside the literal set, a REDUCE on something that is not one of those three
names -- raises ValueError.  Nothing from the file is executed.
"""
import pickletools

import numpy as np

_ALLOWED = {("numpy.core.multiarray", "_reconstruct"): "reconstruct", ("numpy", "ndarray"): "ndarray",
            ("numpy", "dtype"): "dtype", ("numpy._core.multiarray", "_reconstruct"): "reconstruct"}


class _Name:
    def __init__(self, kind):
        self.kind = kind


class _Arr:
    """An ndarray under construction: _reconstruct(...) then BUILD(state)."""

    def __init__(self):
        self.value = None

    def build(self, state):
        _version, shape, dt, fortran, raw = state
        if not isinstance(dt, np.dtype):
            raise ValueError("array state without a dtype")
        if dt == np.dtype(object):
            if not isinstance(raw, list):
                raise ValueError("object array state must be a list")
            a = np.empty(len(raw), dtype=object)
            for i, v in enumerate(raw):
                a[i] = v
            self.value = a.reshape(shape)
            return
        if not isinstance(raw, (bytes, bytearray)):
            raise ValueError("numeric array state must carry raw bytes")
        a = np.frombuffer(bytes(raw), dtype=dt).copy()
        self.value = a.reshape(shape, order="F" if fortran else "C")


class _Dt:
    def __init__(self, descr):
        self.descr = descr
        self.value = None

    def build(self, state):
        order = state[1]
        dt = np.dtype(self.descr)
        if order in ("<", ">"):
            dt = dt.newbyteorder(order)
        self.value = dt


def _resolve(v):
    if isinstance(v, (_Arr, _Dt)):
        return v.value
    if isinstance(v, tuple):
        return tuple(_resolve(x) for x in v)
    if isinstance(v, list):
        return [_resolve(x) for x in v]
    if isinstance(v, dict):
        return {k: _resolve(x) for k, x in v.items()}
    return v


def parse_pickled_npy(path):
    """The object stored by np.save of a dict of arrays, rebuilt from its pickle tokens."""
    with open(path, "rb") as fh:
        version = np.lib.format.read_magic(fh)
        shape, _fortran, dtype = np.lib.format._read_array_header(fh, version)
        if dtype != np.dtype(object) or shape != ():
            raise ValueError(f"{path}: not a 0-d object array")
        data = fh.read()
    stack, memo, marks = [], {}, []
    result = None
    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n == "PROTO":
            continue
        elif n in ("GLOBAL", "STACK_GLOBAL"):
            if n == "STACK_GLOBAL":
                name = stack.pop()
                mod = stack.pop()
            else:
                mod, name = arg.split(" ", 1)
            kind = _ALLOWED.get((mod, name))
            if kind is None:
                raise ValueError(f"{path}: refuses global {mod}.{name}")
            stack.append(_Name(kind))
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n in ("BININT", "BININT1", "BININT2", "BINFLOAT", "SHORT_BINBYTES", "BINBYTES", "BINUNICODE",
                   "SHORT_BINUNICODE", "BINUNICODE8", "BINBYTES8"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "MARK":
            marks.append(len(stack))
        elif n == "TUPLE":
            m = marks.pop()
            items = tuple(stack[m:])
            del stack[m:]
            stack.append(items)
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "APPENDS":
            m = marks.pop()
            items = stack[m:]
            del stack[m:]
            stack[-1].extend(items)
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "SETITEMS":
            m = marks.pop()
            items = stack[m:]
            del stack[m:]
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "REDUCE":
            args = stack.pop()
            f = stack.pop()
            if not isinstance(f, _Name):
                raise ValueError(f"{path}: REDUCE on a non-whitelisted callable")
            if f.kind == "reconstruct":
                if not (isinstance(args, tuple) and len(args) == 3 and isinstance(args[0], _Name)
                        and args[0].kind == "ndarray"):
                    raise ValueError(f"{path}: unexpected _reconstruct arguments")
                stack.append(_Arr())
            elif f.kind == "dtype":
                if not (isinstance(args, tuple) and isinstance(args[0], str)):
                    raise ValueError(f"{path}: unexpected dtype arguments")
                stack.append(_Dt(args[0]))
            else:
                raise ValueError(f"{path}: REDUCE on {f.kind}")
        elif n == "BUILD":
            state = _resolve(stack.pop())
            obj = stack[-1]
            if not isinstance(obj, (_Arr, _Dt)):
                raise ValueError(f"{path}: BUILD on an unexpected object")
            obj.build(state)
        elif n == "STOP":
            result = _resolve(stack.pop())
            break
        else:
            raise ValueError(f"{path}: opcode {n} outside the literal set")
    if not isinstance(result, np.ndarray) or result.shape != ():
        raise ValueError(f"{path}: expected a 0-d object array")
    obj = result.item() if result.dtype == object else result
    if not isinstance(obj, dict):
        raise ValueError(f"{path}: expected a dict")
    return obj
