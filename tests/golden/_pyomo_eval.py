"""Numeric stand-in for the slice of Pyomo that the reference FTE (`src/core/fte.py`) uses.

Used ONLY by `make_golden.py` (in the build container) to run the reference's own
`core.fte.fte` model construction, because Pyomo and IPOPT are not installed. It does
not solve anything. It lets the reference build its model exactly as written
(`src/core/fte.py:176-510`: sets, params, variables with their initial values, the
constraint rules and the objective rule) and then EVALUATES those rules at chosen
variable values:

* every equality constraint `lhs == rhs` evaluates to its residual lhs - rhs;
* a ranged constraint `(lo, e, hi)` to the value of e and its bounds;
* an inequality `e <= c` to e - c (violated when > 0);
* the objective rule to its value.

`SolverFactory('ipopt').solve(m)` calls `SOLVE_HOOK(m)` instead of IPOPT; the fixture
script uses it to record the reference's initial point, evaluate the model at feasible
points it builds, and leave the variables at one of them so the reference's own
post-processing (states, marker positions, reprojection table) runs on it.
"""
import math

import numpy as np

SOLVE_HOOK = None


def _val(o):
    return o._value() if isinstance(o, _Arith) else o


class _Arith:
    """Numeric value with Pyomo-style relational operators."""
    __array_ufunc__ = None       # numpy scalars defer to our reflected operators
    __hash__ = object.__hash__

    def _value(self):
        raise NotImplementedError

    def __float__(self):
        return float(self._value())

    def __add__(self, o):
        return Num(self._value() + _val(o))

    def __radd__(self, o):
        return Num(_val(o) + self._value())

    def __sub__(self, o):
        return Num(self._value() - _val(o))

    def __rsub__(self, o):
        return Num(_val(o) - self._value())

    def __mul__(self, o):
        return Num(self._value() * _val(o))

    def __rmul__(self, o):
        return Num(_val(o) * self._value())

    def __truediv__(self, o):
        return Num(self._value() / _val(o))

    def __rtruediv__(self, o):
        return Num(_val(o) / self._value())

    def __pow__(self, o):
        return Num(self._value() ** _val(o))

    def __rpow__(self, o):
        return Num(_val(o) ** self._value())

    def __neg__(self):
        return Num(-self._value())

    def __pos__(self):
        return Num(self._value())

    def __abs__(self):
        return Num(abs(self._value()))

    def __eq__(self, o):
        return Relation('==', self._value() - _val(o))

    def __le__(self, o):
        return Relation('<=', self._value() - _val(o))

    def __ge__(self, o):
        return Relation('<=', _val(o) - self._value())

    __lt__ = __le__
    __gt__ = __ge__


class Num(_Arith):
    __slots__ = ('v',)

    def __init__(self, v):
        self.v = float(v)

    def _value(self):
        return self.v


class VarData(_Arith):
    __slots__ = ('value',)

    def __init__(self, value=None):
        self.value = value

    def _value(self):
        if self.value is None:
            raise ValueError('variable without a value used in an expression')
        return float(self.value)


class Relation:
    """Evaluated constraint body: kind '==' (residual) or '<=' (e - bound)."""
    __slots__ = ('kind', 'value')

    def __init__(self, kind, value):
        self.kind, self.value = kind, float(value)

    def __bool__(self):
        raise TypeError('relation used as a boolean')


def _fn(f):
    def g(x):
        return Num(f(x._value())) if isinstance(x, _Arith) else f(x)
    g.__name__ = f.__name__
    return g


sin, cos, tan = _fn(math.sin), _fn(math.cos), _fn(math.tan)
atan, sqrt, exp, log = _fn(math.atan), _fn(math.sqrt), _fn(math.exp), _fn(math.log)


class RangeSet:
    def __init__(self, n):
        self.n = int(n)

    def __iter__(self):
        return iter(range(1, self.n + 1))

    def __len__(self):
        return self.n


def _keys(sets):
    if not sets:
        return [None]
    grids = np.meshgrid(*[np.arange(1, len(s) + 1) for s in sets], indexing='ij')
    flat = [g.ravel().tolist() for g in grids]
    if len(sets) == 1:
        return flat[0]
    return list(zip(*flat))


class _Component:
    name = None

    def _construct(self, model, name):
        self.name = name


class _Indexed(_Component):
    def __init__(self, *sets, **kw):
        self.sets, self.kw, self.data = sets, kw, {}

    def __getitem__(self, k):
        return self.data[k]

    def keys(self):
        return list(self.data.keys())


class Param(_Indexed):
    def _construct(self, model, name):
        super()._construct(model, name)
        init = self.kw.get('initialize')
        for k in _keys(self.sets):
            args = k if isinstance(k, tuple) else (k,)
            self.data[k] = float(init(model, *args)) if callable(init) else float(init)


class Var(_Indexed):
    def _construct(self, model, name):
        super()._construct(model, name)
        init = self.kw.get('initialize')
        for k in _keys(self.sets):
            self.data[k] = VarData(init)

    def values(self):
        return np.array([np.nan if d.value is None else float(d.value) for d in self.data.values()])

    def set_values(self, arr):
        arr = np.asarray(arr, np.float64).ravel()
        assert arr.size == len(self.data)
        for d, v in zip(self.data.values(), arr):
            d.value = float(v)


class Constraint(_Indexed):
    Skip = object()

    def __init__(self, *sets, rule=None, **kw):
        super().__init__(*sets, **kw)
        self.rule = rule

    def evaluate(self, model):
        """{key: ('==', residual) | ('<=', e - c) | ('range', lo, e, hi)} of every index."""
        out = {}
        for k in _keys(self.sets):
            args = k if isinstance(k, tuple) else (k,)
            r = self.rule(model, *args)
            if r is Constraint.Skip:
                continue
            if isinstance(r, tuple):
                lo, e, hi = r
                out[k] = ('range', _val(lo), _val(e), _val(hi))
            elif isinstance(r, Relation):
                out[k] = (r.kind, r.value)
            else:
                raise TypeError(f'constraint {self.name}[{k}] evaluated to {r!r}')
        return out


class Objective(_Component):
    def __init__(self, rule=None, **kw):
        self.rule = rule

    def evaluate(self, model):
        return float(_val(self.rule(model)))


class ConcreteModel:
    def __init__(self, name=''):
        object.__setattr__(self, '_components', {})
        object.__setattr__(self, 'name', name)

    def __setattr__(self, name, value):
        if isinstance(value, _Component):
            value._construct(self, name)
            self._components[name] = value
        object.__setattr__(self, name, value)

    def components(self, kind):
        return {k: v for k, v in self._components.items() if isinstance(v, kind)}


class _Solver:
    def __init__(self, name, **kw):
        self.name, self.kw, self.options = name, kw, {}

    def solve(self, model, tee=False, **kw):
        if SOLVE_HOOK is None:
            raise RuntimeError('no IPOPT here: set _pyomo_eval.SOLVE_HOOK')
        return SOLVE_HOOK(model)


def SolverFactory(name, **kw):
    return _Solver(name, **kw)


def install():
    """Register this module as `pyomo`, `pyomo.environ` and `pyomo.opt`."""
    import sys
    import types
    me = sys.modules[__name__]
    pkg = types.ModuleType('pyomo')
    pkg.environ = me
    opt = types.ModuleType('pyomo.opt')
    opt.SolverFactory = SolverFactory
    pkg.opt = opt
    sys.modules['pyomo'] = pkg
    sys.modules['pyomo.environ'] = me
    sys.modules['pyomo.opt'] = opt
