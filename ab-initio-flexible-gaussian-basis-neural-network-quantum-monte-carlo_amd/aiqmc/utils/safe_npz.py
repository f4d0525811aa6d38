"""Weights-only reader for the reference's checkpoint files (AIQMCrelease3/checkpoint.py:44-70).

The reference saves ``np.savez(t=..., data=asdict(AINetData), params=<pytree>, opt_state=...)``:
``params`` / ``data`` / ``opt_state`` become 0-d object arrays whose payload is a pickle
stream of JAX arrays (``jax._src.array._reconstruct_array(fun, args, arr_state,
aval_state)`` wrapping numpy's ``_reconstruct`` + ``__setstate__``), numpy scalars and,
for ``opt_state``, optax NamedTuple states.  ``np.load(allow_pickle=True)`` would import
and call whatever the stream names.  This module never unpickles: it walks the stream's
opcodes with ``pickletools.genops`` (a tokenizer -- it executes nothing) and builds the
result itself from a fixed vocabulary:

* containers: dict / list / tuple / memo references;
* numpy arrays: only the ``_reconstruct`` + BUILD(state) pattern, materialised with
  ``np.frombuffer`` (numeric dtypes) or from the element list (object dtype);
* ``numpy.dtype(spec, align, copy)`` + BUILD(byte order), numpy ``scalar(dtype, bytes)``;
* JAX ``_reconstruct_array`` -> the numpy array it wraps (device placement dropped);
* ``collections.OrderedDict`` -> dict;
* optax state NamedTuples (``RECORD_TYPES``) -> :class:`Record` (name + fields, tuple-like);
* kfac_jax optimizer states (``main/main_pp.py`` checkpoints ``opt_state`` of
  ``kfac_jax.Optimizer``; every release2/release3 checkpoint the reference ships holds one):
  the stream names the state class as ``builtins.getattr(<class>, "State")`` and builds it by
  ``NEWOBJ(cls, ())`` + ``BUILD(field dict)``.  ``getattr`` is accepted only as that exact
  pattern -- a class marker from ``STATE_OWNERS`` and the literal attribute ``"State"`` --
  and yields another marker, never an attribute lookup; the object becomes a
  :class:`StateRecord` (class name + field dict) and nothing else.  ``STATE_TYPES`` lists
  the dataclasses built directly (``WeightedMovingAverage``).

Any other global, an opcode outside the vocabulary, or a self-referential container raises
:class:`UnsafeCheckpointError`.
"""
from __future__ import annotations

import io
import pickletools
import zipfile
from typing import Any, Dict, List, Tuple

import numpy as np
from numpy.lib import format as npformat

__all__ = ["UnsafeCheckpointError", "Record", "StateRecord", "load_npz", "loads_pickle_stream", "RECORD_TYPES",
           "STATE_OWNERS", "STATE_TYPES"]


class UnsafeCheckpointError(ValueError):
    """The file holds something outside the weights-only vocabulary."""


class Record(tuple):
    """A NamedTuple from the stream (optax states): tuple of fields + the original class name."""

    def __new__(cls, name: str, fields):
        obj = super().__new__(cls, tuple(fields))
        obj.type_name = name
        return obj

    def __repr__(self):
        return f"Record({self.type_name}, {tuple(self)!r})"


class StateRecord(dict):
    """A dataclass state from the stream (kfac_jax): field dict + the original class name.
    Fields read as items or attributes (``rec["velocities"]`` / ``rec.velocities``)."""

    def __init__(self, name: str, fields: Dict[str, Any]):
        super().__init__(fields)
        self.type_name = name

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __repr__(self):
        return f"StateRecord({self.type_name}, {dict.__repr__(self)})"


# NamedTuple classes of the optimizer states the drivers checkpoint (optax chain of
# scale_by_adam / scale_by_schedule / scale, main_all_electrons_adam_muti_GPU.py:152-158).
RECORD_TYPES = {
    "optax._src.transform ScaleByAdamState",
    "optax._src.transform ScaleByScheduleState",
    "optax._src.transform ScaleState",
    "optax._src.base EmptyState",
    "optax._src.transform ScaleByRmsState",
    "optax._src.transform TraceState",
}
# Classes whose nested ``State`` dataclass may be named through getattr(<class>, "State")
# (kfac_jax 0.0.x: optimizer, curvature estimator and the curvature blocks the network's
# layers map to; the reference's KFAC driver registers dense and scale-and-shift blocks,
# Optimizer/curvature_tags_and_blocks.py).
STATE_OWNERS = {
    "kfac_jax._src.optimizer Optimizer",
    "kfac_jax._src.curvature_estimator BlockDiagonalCurvature",
    "kfac_jax._src.curvature_blocks Diagonal",
    "kfac_jax._src.curvature_blocks Full",
    "kfac_jax._src.curvature_blocks KroneckerFactored",
    "kfac_jax._src.curvature_blocks TwoKroneckerFactored",
    "kfac_jax._src.curvature_blocks ScaleAndShiftDiagonal",
    "kfac_jax._src.curvature_blocks ScaleAndShiftFull",
}
# Dataclasses built directly by NEWOBJ(cls, ()) + BUILD(fields).
STATE_TYPES = {
    "kfac_jax._src.utils.accumulators WeightedMovingAverage",
}
_NUMPY_MODULES = ("numpy.core.multiarray", "numpy._core.multiarray")


class _Marker:
    def __init__(self, name: str):
        self.name = name


class _DType:
    """A dtype under construction (BUILD may set its byte order)."""

    def __init__(self, spec: str):
        try:
            self.dtype = np.dtype(spec)
        except TypeError as e:
            raise UnsafeCheckpointError(f"dtype {spec!r}") from e

    def build(self, state):
        if isinstance(state, tuple) and len(state) >= 2 and state[1] in ("<", ">", "|", "=") \
                and self.dtype.kind not in ("O", "V"):
            self.dtype = self.dtype.newbyteorder(state[1]) if state[1] in "<>" else self.dtype


class _Object:
    """A STATE_TYPES / <owner>.State object under construction: BUILD fills its fields."""

    def __init__(self, name: str):
        self.name = name
        self.fields: Dict[str, Any] = {}

    def build(self, state):
        # object.__reduce_ex__ state: the instance dict, or (dict | None, slots dict | None).
        parts = state if isinstance(state, tuple) and len(state) == 2 else (state,)
        for part in parts:
            if part is None:
                continue
            if not isinstance(part, dict) or not all(isinstance(k, str) for k in part):
                raise UnsafeCheckpointError(f"unexpected state of {self.name}")
            self.fields.update(part)


class _Array:
    """numpy ``_reconstruct(ndarray, shape, b'b')``; BUILD((ver, shape, dtype, fortran, raw))."""

    def __init__(self):
        self.value = None

    def build(self, state):
        if not (isinstance(state, tuple) and len(state) == 5):
            raise UnsafeCheckpointError("unexpected ndarray state")
        _, shape, dt, fortran, raw = state
        if not isinstance(dt, _DType):
            raise UnsafeCheckpointError("ndarray state without a dtype")
        shape = tuple(int(s) for s in shape)
        order = "F" if fortran else "C"
        if dt.dtype.hasobject:
            if not isinstance(raw, list):
                raise UnsafeCheckpointError("object array without an element list")
            arr = np.empty(len(raw), dtype=object)
            for k, v in enumerate(raw):
                arr[k] = v
            self.value = arr.reshape(shape, order=order)
        else:
            if not isinstance(raw, (bytes, bytearray)):
                raise UnsafeCheckpointError("numeric array without raw bytes")
            self.value = np.frombuffer(bytes(raw), dtype=dt.dtype).reshape(shape, order=order).copy()


def _global(module: str, name: str):
    full = f"{module} {name}"
    if module in _NUMPY_MODULES and name == "_reconstruct":
        return _Marker("ndarray_reconstruct")
    if module in _NUMPY_MODULES and name == "scalar":
        return _Marker("scalar")
    if module == "numpy" and name == "ndarray":
        return _Marker("ndarray")
    if module == "numpy" and name == "dtype":
        return _Marker("dtype")
    if module.startswith("jax") and name == "_reconstruct_array":
        return _Marker("jax_array")
    if module == "collections" and name == "OrderedDict":
        return _Marker("odict")
    if full in RECORD_TYPES:
        return _Marker("record:" + full)
    if module == "builtins" and name == "getattr":
        return _Marker("getattr")
    if full in STATE_OWNERS:
        return _Marker("owner:" + full)
    if full in STATE_TYPES:
        return _Marker("state:" + full)
    raise UnsafeCheckpointError(f"refusing global {module}.{name}")


def _call(fn, args: tuple):
    if not isinstance(fn, _Marker):
        raise UnsafeCheckpointError("call of a non-global")
    k = fn.name
    if k == "ndarray_reconstruct":
        if not (len(args) == 3 and isinstance(args[0], _Marker) and args[0].name == "ndarray"):
            raise UnsafeCheckpointError("unexpected _reconstruct arguments")
        return _Array()
    if k == "dtype":
        if not args or not isinstance(args[0], str):
            raise UnsafeCheckpointError("unexpected dtype arguments")
        return _DType(args[0])
    if k == "scalar":
        dt, raw = args[0], args[1] if len(args) > 1 else None
        if not isinstance(dt, _DType) or not isinstance(raw, (bytes, bytearray)) or dt.dtype.hasobject:
            raise UnsafeCheckpointError("unexpected numpy scalar")
        return np.frombuffer(bytes(raw), dtype=dt.dtype)[0]
    if k == "jax_array":
        fun, fargs, arr_state = args[0], args[1], args[2]
        a = _call(fun, tuple(fargs))
        if not isinstance(a, _Array):
            raise UnsafeCheckpointError("jax array without a numpy payload")
        a.build(arr_state)
        return a.value
    if k == "odict":
        d: Dict[Any, Any] = {}
        for kv in (args[0] if args else []):
            d[kv[0]] = kv[1]
        return d
    if k.startswith("record:"):
        return Record(k[len("record:"):].split(" ")[1], args)
    if k == "getattr":
        if not (len(args) == 2 and isinstance(args[0], _Marker) and args[0].name.startswith("owner:")
                and isinstance(args[1], str) and args[1] == "State"):
            raise UnsafeCheckpointError("getattr outside the <kfac class>.State pattern")
        return _Marker("state:" + args[0].name[len("owner:"):] + ".State")
    raise UnsafeCheckpointError(f"cannot call {k}")


def _newobj(cls, args: tuple):
    """NEWOBJ: namedtuple records (cls(*fields)) or an empty state object filled by BUILD."""
    if isinstance(cls, _Marker) and cls.name.startswith("state:"):
        if args:
            raise UnsafeCheckpointError(f"unexpected constructor arguments for {cls.name}")
        mod_cls = cls.name[len("state:"):].split(" ", 1)[1]
        return _Object(mod_cls)
    return _call(cls, args)


_IN_PROGRESS = object()


def _resolve(obj, seen=None):
    """Replace the construction helpers by their values.  Mutable containers are registered
    before their children are visited (a memo reference back to them resolves to the same
    object); an immutable one reached again while it is being resolved is a cycle that a
    weights-only file never holds, and is refused."""
    if seen is None:
        seen = {}
    oid = id(obj)
    if oid in seen:
        if seen[oid] is _IN_PROGRESS:
            raise UnsafeCheckpointError("self-referential object in the stream")
        return seen[oid]
    if isinstance(obj, dict) and not isinstance(obj, StateRecord):
        out = {}
        seen[oid] = out
        for k, v in obj.items():
            out[_resolve(k, seen)] = _resolve(v, seen)
        return out
    if isinstance(obj, list):
        out = []
        seen[oid] = out
        out.extend(_resolve(v, seen) for v in obj)
        return out
    seen[oid] = _IN_PROGRESS
    if isinstance(obj, _Array):
        if obj.value is None:
            raise UnsafeCheckpointError("ndarray never built")
        out = obj.value
        if out.dtype.hasobject:
            flat = out.reshape(-1)
            for i in range(flat.size):
                flat[i] = _resolve(flat[i], seen)
    elif isinstance(obj, _DType):
        out = obj.dtype
    elif isinstance(obj, _Object):
        out = StateRecord(obj.name, {k: _resolve(v, seen) for k, v in obj.fields.items()})
    elif isinstance(obj, Record):
        out = Record(obj.type_name, [_resolve(v, seen) for v in obj])
    elif isinstance(obj, tuple):
        out = tuple(_resolve(v, seen) for v in obj)
    elif isinstance(obj, np.ndarray) and obj.dtype.hasobject:
        out = np.empty(obj.shape, dtype=object)
        for idx in np.ndindex(obj.shape):
            out[idx] = _resolve(obj[idx], seen)
    elif isinstance(obj, _Marker):
        raise UnsafeCheckpointError(f"dangling global {obj.name}")
    else:
        out = obj
    seen[oid] = out
    return out


_PUSH_CONST = {"NONE": None, "NEWTRUE": True, "NEWFALSE": False}
_PUSH_ARG = {"BININT", "BININT1", "BININT2", "LONG1", "LONG4", "BINFLOAT", "BINUNICODE", "SHORT_BINUNICODE",
             "BINUNICODE8", "BINBYTES", "SHORT_BINBYTES", "BINBYTES8", "UNICODE", "INT", "LONG", "FLOAT",
             "STRING", "BINSTRING", "SHORT_BINSTRING"}


def loads_pickle_stream(data: bytes):
    """Interpret a pickle stream from the weights-only vocabulary; nothing is imported or called."""
    stack: List[Any] = []
    marks: List[int] = []
    memo: Dict[int, Any] = {}

    def pop_mark() -> List[Any]:
        if not marks:
            raise UnsafeCheckpointError("MARK underflow")
        m = marks.pop()
        items = stack[m:]
        del stack[m:]
        return items

    for op, arg, _ in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            if len(stack) != 1:
                raise UnsafeCheckpointError("malformed stream")
            try:
                return _resolve(stack[0])
            except RecursionError as e:
                raise UnsafeCheckpointError("object nesting too deep") from e
        if n in _PUSH_CONST:
            stack.append(_PUSH_CONST[n])
        elif n in _PUSH_ARG:
            if n in ("STRING", "BINSTRING", "SHORT_BINSTRING") and isinstance(arg, bytes):
                arg = arg.decode("latin-1")
            stack.append(arg)
        elif n == "BYTEARRAY8":
            stack.append(bytearray(arg))
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "MARK":
            marks.append(len(stack))
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == "LIST":
            stack.append(list(pop_mark()))
        elif n == "DICT":
            items = pop_mark()
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif n == "APPEND":
            v = stack.pop()
            if not isinstance(stack[-1], list):
                raise UnsafeCheckpointError("APPEND to a non-list")
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            if not isinstance(stack[-1], list):
                raise UnsafeCheckpointError("APPENDS to a non-list")
            stack[-1].extend(items)
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            if not isinstance(stack[-1], dict):
                raise UnsafeCheckpointError("SETITEM on a non-dict")
            stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            if not isinstance(stack[-1], dict):
                raise UnsafeCheckpointError("SETITEMS on a non-dict")
            for i in range(0, len(items), 2):
                stack[-1][items[i]] = items[i + 1]
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[int(arg)] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[int(arg)])
        elif n == "GLOBAL":
            module, name = arg.split(" ", 1)
            stack.append(_global(module, name))
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            module = stack.pop()
            stack.append(_global(str(module), str(name)))
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(_call(fn, tuple(args)))
        elif n == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(_newobj(cls, tuple(args)))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, (_Array, _DType, _Object)):
                obj.build(state)
            elif isinstance(obj, dict) and isinstance(state, dict):
                obj.update(state)
            else:
                raise UnsafeCheckpointError(f"BUILD on {type(obj).__name__}")
        else:
            raise UnsafeCheckpointError(f"opcode {n} is outside the weights-only vocabulary")
    raise UnsafeCheckpointError("stream without STOP")


def _read_npy(raw: bytes):
    f = io.BytesIO(raw)
    version = npformat.read_magic(f)
    if version == (1, 0):
        shape, fortran, dtype = npformat.read_array_header_1_0(f)
    elif version in ((2, 0), (3, 0)):
        shape, fortran, dtype = npformat.read_array_header_2_0(f)
    else:
        raise UnsafeCheckpointError(f"npy version {version}")
    body = f.read()
    if dtype.hasobject:
        arr = loads_pickle_stream(body)
        if not isinstance(arr, np.ndarray):
            arr = np.asarray(arr, dtype=object)
        return arr
    n = int(np.prod(shape)) if shape else 1
    a = np.frombuffer(body[:n * dtype.itemsize], dtype=dtype)
    return a.reshape(shape, order="F" if fortran else "C").copy()


def load_npz(path_or_file) -> Dict[str, np.ndarray]:
    """All members of an .npz as numpy arrays, object members decoded by the weights-only
    interpreter (a 0-d object array whose ``.item()`` is the saved pytree)."""
    out: Dict[str, np.ndarray] = {}
    with zipfile.ZipFile(path_or_file) as z:
        for info in z.infolist():
            key = info.filename[:-4] if info.filename.endswith(".npy") else info.filename
            out[key] = _read_npy(z.read(info))
    return out
