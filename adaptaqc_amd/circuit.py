"""Minimal quantum-circuit IR standing in for the parts of ``qiskit.QuantumCircuit`` that the
hot path touches (qiskit is not a dependency here).

Mirrors the attribute shapes the reference code reads: ``circuit.data[i].operation.name /
.params / .label``, ``circuit.data[i].qubits``, ``num_qubits``, ``copy()``, ``inverse()``,
``compose(other, qubits)`` and ``set_matrix_product_state(mps)``
(approximate_compiler.py:180-204).  Qubits are plain integers (little-endian: qubit 0 is the
least significant bit of a statevector index).
"""
from __future__ import annotations

import numpy as np

from . import gates as G

ONE_Q = set(G.CONST_1Q) | {"rx", "ry", "rz", "p", "u1", "u", "u3", "u2"}
TWO_Q = set(G.TWO_QUBIT) | {"crx", "cry", "crz", "cp", "cu1", "rzz"}
_SELF_INVERSE = {"id", "x", "y", "z", "h", "cx", "cy", "cz", "swap", "ccx"}
_INVERSE_NAME = {"s": "sdg", "sdg": "s", "t": "tdg", "tdg": "t", "sx": "sxdg", "sxdg": "sx"}
_PARAM_NEGATE = {"rx", "ry", "rz", "p", "u1", "crx", "cry", "crz", "cp", "cu1", "rzz"}


class Operation:
    """A named gate (``qiskit.circuit.Gate`` stand-in)."""

    __slots__ = ("name", "params", "label", "num_qubits")

    def __init__(self, name, num_qubits, params=(), label=None):
        self.name = name
        self.num_qubits = num_qubits
        self.params = list(params)
        self.label = label

    def copy(self):
        return Operation(self.name, self.num_qubits, list(self.params), self.label)

    def to_matrix(self):
        if self.name == "unitary":
            return np.asarray(self.params[0], dtype=complex)
        if self.num_qubits == 1:
            return G.one_qubit(self.name, self.params)
        if self.num_qubits == 2:
            return G.two_qubit(self.name, self.params)
        raise ValueError(f"no matrix for {self.name}")

    def inverse(self):
        if self.name in _SELF_INVERSE:
            return self.copy()
        if self.name in _INVERSE_NAME:
            return Operation(_INVERSE_NAME[self.name], self.num_qubits, (), self.label)
        if self.name in _PARAM_NEGATE:
            return Operation(self.name, self.num_qubits, [-p for p in self.params], self.label)
        if self.name in ("u", "u3"):
            t, ph, lam = self.params
            return Operation(self.name, 1, [-t, -lam, -ph], self.label)
        if self.name == "u2":
            ph, lam = self.params
            return Operation("u3", 1, [-np.pi / 2, -lam, -ph], self.label)
        if self.name == "unitary":
            return Operation("unitary", self.num_qubits, [np.conj(np.asarray(self.params[0])).T], self.label)
        raise ValueError(f"cannot invert {self.name}")

    def _key(self):
        ps = []
        for p in self.params:
            if isinstance(p, np.ndarray):
                ps.append(("arr", p.shape, p.tobytes()))
            elif isinstance(p, tuple) and self.name == "set_matrix_product_state":
                ps.append(("mps", id(p)))
            else:
                ps.append(float(p) if np.isscalar(p) else p)
        return (self.name, tuple(ps))

    def __eq__(self, other):
        return isinstance(other, Operation) and self._key() == other._key()

    def __repr__(self):
        return f"Operation({self.name!r}, params={self.params})"


class CircuitInstruction:
    __slots__ = ("operation", "qubits", "clbits")

    def __init__(self, operation, qubits, clbits=()):
        self.operation = operation
        self.qubits = tuple(int(q) for q in qubits)
        self.clbits = tuple(clbits)

    def copy(self):
        return CircuitInstruction(self.operation.copy(), self.qubits, self.clbits)

    def __eq__(self, other):
        return (
            isinstance(other, CircuitInstruction)
            and self.qubits == other.qubits
            and self.operation == other.operation
        )

    def __iter__(self):  # legacy (instr, qargs, cargs) unpacking
        return iter((self.operation, self.qubits, self.clbits))


class QuantumCircuit:
    def __init__(self, num_qubits: int):
        self.num_qubits = int(num_qubits)
        self.data: list[CircuitInstruction] = []

    # -- construction ------------------------------------------------------------------
    def append(self, operation, qubits):
        qubits = tuple(int(q) for q in (qubits if np.iterable(qubits) else [qubits]))
        for q in qubits:
            if not 0 <= q < self.num_qubits:
                raise IndexError(f"qubit {q} out of range for {self.num_qubits}-qubit circuit")
        if len(set(qubits)) != len(qubits):
            raise ValueError("duplicate qubit arguments")
        self.data.append(CircuitInstruction(operation, qubits))
        return self

    def _g1(self, name, qubit, params=(), label=None):
        for q in (qubit if np.iterable(qubit) else [qubit]):
            self.append(Operation(name, 1, params, label), [q])
        return self

    def rx(self, theta, q):
        return self._g1("rx", q, [theta])

    def ry(self, theta, q):
        return self._g1("ry", q, [theta])

    def rz(self, theta, q):
        return self._g1("rz", q, [theta])

    def p(self, lam, q):
        return self._g1("p", q, [lam])

    def u(self, theta, phi, lam, q):
        return self._g1("u", q, [theta, phi, lam])

    def x(self, q):
        return self._g1("x", q)

    def y(self, q):
        return self._g1("y", q)

    def z(self, q):
        return self._g1("z", q)

    def h(self, q):
        return self._g1("h", q)

    def s(self, q):
        return self._g1("s", q)

    def sdg(self, q):
        return self._g1("sdg", q)

    def t(self, q):
        return self._g1("t", q)

    def tdg(self, q):
        return self._g1("tdg", q)

    def sx(self, q):
        return self._g1("sx", q)

    def id(self, q):
        return self._g1("id", q)

    def cx(self, c, t):
        return self.append(Operation("cx", 2), [c, t])

    def cy(self, c, t):
        return self.append(Operation("cy", 2), [c, t])

    def cz(self, c, t):
        return self.append(Operation("cz", 2), [c, t])

    def swap(self, a, b):
        return self.append(Operation("swap", 2), [a, b])

    def crz(self, theta, c, t):
        return self.append(Operation("crz", 2, [theta]), [c, t])

    def rzz(self, theta, a, b):
        return self.append(Operation("rzz", 2, [theta]), [a, b])

    def ccx(self, a, b, c):
        return self.append(Operation("ccx", 3), [a, b, c])

    def unitary(self, matrix, qubits, label=None):
        qubits = list(qubits) if np.iterable(qubits) else [qubits]
        m = np.asarray(matrix, dtype=complex)
        if m.shape != (2 ** len(qubits),) * 2:
            raise ValueError("unitary shape does not match qubit count")
        return self.append(Operation("unitary", len(qubits), [m], label), qubits)

    def set_matrix_product_state(self, mps):
        """Embed an Aer-format MPS (list[(G0, G1)], list[lambda]) as the initial state."""
        gam, lam = mps
        if len(gam) != self.num_qubits:
            raise ValueError("MPS size does not match the circuit")
        op = Operation("set_matrix_product_state", self.num_qubits, [mps])
        self.data.append(CircuitInstruction(op, range(self.num_qubits)))
        return self

    def barrier(self, *args):
        return self

    def find_bit(self, q):
        """qiskit's ``find_bit``: here qubits are their own indices."""
        return BitLocation(int(q))

    # -- container protocol ------------------------------------------------------------
    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(self.data)

    def __getitem__(self, i):
        return self.data[i]

    def __eq__(self, other):
        return (
            isinstance(other, QuantumCircuit)
            and self.num_qubits == other.num_qubits
            and len(self.data) == len(other.data)
            and all(a == b for a, b in zip(self.data, other.data))
        )

    def __repr__(self):
        body = ", ".join(f"{i.operation.name}{list(i.qubits)}" for i in self.data[:12])
        more = "" if len(self.data) <= 12 else f", ... (+{len(self.data) - 12})"
        return f"QuantumCircuit({self.num_qubits}: {body}{more})"

    def copy(self):
        qc = QuantumCircuit(self.num_qubits)
        qc.data = [i.copy() for i in self.data]
        return qc

    def inverse(self):
        qc = QuantumCircuit(self.num_qubits)
        for ins in reversed(self.data):
            if ins.operation.name == "set_matrix_product_state":
                raise ValueError("cannot invert a circuit holding an MPS state")
            qc.data.append(CircuitInstruction(ins.operation.inverse(), ins.qubits))
        return qc

    def compose(self, other, qubits=None):
        """Return self followed by ``other`` mapped onto ``qubits`` (qiskit semantics)."""
        qc = self.copy()
        mapping = list(range(other.num_qubits)) if qubits is None else list(qubits)
        for ins in other.data:
            qc.data.append(CircuitInstruction(ins.operation.copy(), [mapping[q] for q in ins.qubits]))
        return qc

    def count_ops(self):
        out = {}
        for ins in self.data:
            out[ins.operation.name] = out.get(ins.operation.name, 0) + 1
        return out

    def depth(self, filter_function=None):
        level = [0] * self.num_qubits
        for ins in self.data:
            if filter_function is not None and not filter_function(ins):
                continue
            d = max(level[q] for q in ins.qubits) + 1
            for q in ins.qubits:
                level[q] = d
        return max(level) if level else 0


class BitLocation:
    """``QuantumCircuit.find_bit`` result (qiskit's BitLocations: ``.index``)."""

    __slots__ = ("index",)

    def __init__(self, index):
        self.index = index


def mps_payload(op):
    """The Aer-format MPS ``(list[(G0, G1)], list[lambda])`` held by a set_matrix_product_state
    instruction: ``params[0]`` here and in qiskit-aer's SetMatrixProductState; an instruction that
    carries gammas and lambdas as two parameters is accepted too."""
    ps = list(op.params)
    if len(ps) == 2 and isinstance(ps[0], (list, tuple)) and len(ps[0]) and isinstance(ps[0][0], (list, tuple)):
        return ps[0], ps[1]
    return ps[0]


def qubit_indices(circuit, ins):
    """Integer qubit indices of an instruction: plain ints (this IR), or qiskit ``Qubit`` objects
    resolved through ``circuit.find_bit`` (the reference's qiskit circuits)."""
    out = []
    for q in ins.qubits:
        if isinstance(q, (int, np.integer)):
            out.append(int(q))
        else:
            out.append(int(circuit.find_bit(q).index))
    return tuple(out)


def op_matrix(op):
    """Matrix of a gate: this IR's Operation, or a qiskit-shaped gate (standard names through the
    same gate tables, anything else through its own ``to_matrix()``)."""
    if isinstance(op, Operation):
        return op.to_matrix()
    name = op.name
    params = list(getattr(op, "params", ()))
    try:
        vals = [float(p) for p in params]
        if op.num_qubits == 1 and (name in G.CONST_1Q or name in ONE_Q):
            return G.one_qubit(name, vals)
        if op.num_qubits == 2 and name in TWO_Q:
            return G.two_qubit(name, vals)
    except (TypeError, ValueError, KeyError):
        pass
    return np.asarray(op.to_matrix(), dtype=complex)


def decompose(ins, qubits=None):
    """Yield (matrix, qubits) 1-/2-qubit pieces of an instruction (unroll_to_basis_gates)."""
    op = ins.operation
    q = tuple(qubits) if qubits is not None else tuple(ins.qubits)
    name = op.name
    if name in ("barrier", "measure", "id"):
        return
    if name == "ccx":
        a, b, c = q
        seq = [("h", (c,)), ("cx", (b, c)), ("tdg", (c,)), ("cx", (a, c)), ("t", (c,)), ("cx", (b, c)),
               ("tdg", (c,)), ("cx", (a, c)), ("t", (b,)), ("t", (c,)), ("h", (c,)), ("cx", (a, b)),
               ("t", (a,)), ("tdg", (b,)), ("cx", (a, b))]
        for nm, qq in seq:
            yield (G.one_qubit(nm) if len(qq) == 1 else G.two_qubit(nm)), qq
        return
    if op.num_qubits > 2:
        raise ValueError(f"gate {name} on {op.num_qubits} qubits is not supported")
    yield op_matrix(op), q


def device_ops(circuit, start: int = 0):
    """Flatten gates from ``circuit.data[start:]`` into (matrix, qubits) pairs.  ``circuit`` is
    this IR's QuantumCircuit or a qiskit-shaped one (``data`` of instructions with ``operation``
    and ``qubits``, ``find_bit``), so the backends drop into the reference's own compiler."""
    out = []
    for ins in circuit.data[start:]:
        if ins.operation.name == "set_matrix_product_state":
            raise ValueError("set_matrix_product_state must be the first instruction")
        if ins.operation.name in ("barrier", "measure", "id", "delay"):
            continue
        out.extend(decompose(ins, qubit_indices(circuit, ins)))
    return out


# Per-circuit conversion memo of device_ops_array: the rows of every instruction, reused while the
# instruction is unchanged.  ADAPT-AQC re-evaluates the same circuit with a few angles changed
# (Rotosolve / Rotoselect rewrite one gate's parameters, a layer is appended), so an evaluation
# re-converts only those gates: the whole conversion of a 590-gate 20-qubit circuit was ~7 ms of
# Python per evaluation against ~0.5 ms of GPU time.
_SKIP_NAMES = ("barrier", "measure", "id", "delay")
# keyed by id(circuit) with a weak reference to it (circuits define __eq__, so they do not hash);
# an entry goes when its circuit is collected
_OPS_MEMO = {}


def _memo_get(circuit):
    e = _OPS_MEMO.get(id(circuit))
    if e is not None and e[0]() is circuit:
        return e[1], e[2]
    return None


def _memo_put(circuit, start, entries):
    import weakref

    key = id(circuit)
    try:
        ref = weakref.ref(circuit, lambda _r, key=key: _OPS_MEMO.pop(key, None))
    except TypeError:  # not weak-referenceable: no memo
        return
    _OPS_MEMO[key] = (ref, start, entries)


def _from_tables(op):
    """True when op's matrix comes from the gate tables by (name, params) alone -- this IR's
    Operation, or a qiskit-shaped standard gate -- so equal names and parameters mean equal rows.
    A custom gate's matrix comes from its own to_matrix() / definition, which its name and
    parameters need not determine."""
    if isinstance(op, Operation):
        return True
    name = op.name
    n = getattr(op, "num_qubits", None)
    if name in _SKIP_NAMES or name == "ccx":
        return True
    return (n == 1 and (name in G.CONST_1Q or name in ONE_Q)) or (n == 2 and name in TWO_Q)


def _params_snapshot(op):
    """The gate's parameters as a list for equality checks, or None when they are not plain numbers
    (a unitary's matrix, symbolic parameters) or the matrix does not come from the gate tables
    (a custom gate): such gates are re-converted every time."""
    if not _from_tables(op):
        return None
    ps = list(getattr(op, "params", ()))
    for p in ps:
        if not isinstance(p, (int, float, complex, np.number)):
            return None
    return ps


def device_ops_array(circuit, start: int = 0):
    """``_lib.ops_array(device_ops(circuit, start))``, memoised per circuit: an instruction whose
    operation, parameters and qubits are unchanged since the last call reuses its rows (kept as
    bytes: concatenating structured arrays promotes their fields, ~16 us each).  Changed
    instructions are converted together in one ops_array call."""
    from . import _lib

    data = circuit.data
    prev = _memo_get(circuit)
    old = prev[1] if prev is not None and prev[0] == start else ()
    entries, blocks, pending = [], [], []  # pending: (entry index, [(matrix, qubits), ...])
    for i in range(start, len(data)):
        ins = data[i]
        op = ins.operation
        qs = tuple(ins.qubits)
        k = i - start
        c = old[k] if k < len(old) else None
        if c is not None:
            cop, cps, cqs, cblock = c
            if (cps is not None and cqs == qs
                    and (cop is op or (type(cop) is type(op) and cop.name == op.name))
                    and list(getattr(op, "params", ())) == cps):
                entries.append(c)
                blocks.append(cblock)
                continue
        name = op.name
        if name == "set_matrix_product_state":
            raise ValueError("set_matrix_product_state must be the first instruction")
        entries.append(None)
        blocks.append(b"")
        if name in _SKIP_NAMES:
            entries[-1] = (op, _params_snapshot(op), qs, b"")
        else:
            pending.append((len(entries) - 1, op, qs, list(decompose(ins, qubit_indices(circuit, ins)))))
    if pending:
        rows = _lib.ops_array([piece for _, _, _, pieces in pending for piece in pieces])
        raw = rows.tobytes()
        size, off = _lib.OP_DTYPE.itemsize, 0
        for e, op, qs, pieces in pending:
            block = raw[off:off + size * len(pieces)]
            off += size * len(pieces)
            entries[e] = (op, _params_snapshot(op), qs, block)
            blocks[e] = block
    _memo_put(circuit, start, entries)
    return np.frombuffer(b"".join(blocks), dtype=_lib.OP_DTYPE).copy()


def device_ops_rows(circuit, lo: int, hi: int):
    """The op rows of ``circuit.data[lo:hi]`` cut from the memoised conversion of the whole circuit
    after a leading set_matrix_product_state (device_ops_array): a Rotoselect / Rotosolve visit's
    suffix re-converts only the instructions changed since the previous visit (one gate) instead of
    building every suffix gate's matrix again (~6 us a gate in Python: 0.3 ms a visit at 50 qubits)."""
    from . import _lib

    data = circuit.data
    start = 1 if len(data) and data[0].operation.name == "set_matrix_product_state" else 0
    lo, hi = max(lo, start), min(hi, len(data))
    if hi <= lo:
        return np.zeros(0, dtype=_lib.OP_DTYPE)
    arr = device_ops_array(circuit, start)
    prev = _memo_get(circuit)
    if prev is None or prev[0] != start:  # (not memoisable: convert the range directly)
        return _lib.ops_array(device_ops(_Range(circuit, lo, hi)))
    size = _lib.OP_DTYPE.itemsize
    off = np.cumsum([0] + [len(e[3]) // size for e in prev[1]])
    return arr[off[lo - start]:off[hi - start]]


class _Range:
    """``circuit.data[lo:hi]`` with the circuit's qubit resolution (device_ops' input)."""

    def __init__(self, circuit, lo, hi):
        self.data = circuit.data[lo:hi]
        self.num_qubits = circuit.num_qubits
        self._c = circuit

    def find_bit(self, q):
        return self._c.find_bit(q)


_QASM_NAMES = {"rx", "ry", "rz", "p", "u1", "u", "u3", "u2", "x", "y", "z", "h", "s", "sdg", "t", "tdg", "sx",
               "sxdg", "id", "cx", "cy", "cz", "swap", "crx", "cry", "crz", "cp", "cu1", "rzz", "ccx"}


def u3_params(v):
    """(theta, phi, lam, alpha) with v = exp(i alpha) u3(theta, phi, lam) for a 2x2 unitary."""
    v = np.asarray(v, dtype=complex)
    theta = 2.0 * float(np.arctan2(abs(v[1, 0]), abs(v[0, 0])))
    if abs(v[0, 0]) > 1e-12:
        alpha = float(np.angle(v[0, 0]))
        phi = float(np.angle(v[1, 0])) - alpha if abs(v[1, 0]) > 1e-12 else 0.0
        lam = float(np.angle(v[1, 1])) - alpha - phi if abs(v[1, 0]) <= 1e-12 else float(np.angle(-v[0, 1])) - alpha
    else:  # theta = pi: only the off-diagonal is set; phi absorbs the phase
        alpha, phi = float(np.angle(v[1, 0])), 0.0
        lam = float(np.angle(-v[0, 1])) - alpha
    return theta, phi, lam, alpha


def unroll_two_qubit(u):
    """Standard-gate pieces of a 4x4 unitary on local qubits (0, 1) (index 2*b1 + b0, gates.py), up
    to a global phase: the cosine-sine split U = (A0 (+) A1) CS (B0 (+) B1) over bit 1, each
    block-diagonal factor as u3 on qubit 0 then controlled-u3 from qubit 1 (with the control's u1
    phase), and CS as ry on qubit 1 plus cry from qubit 0.  [(name, params, local qubits)]."""
    from scipy.linalg import cossin

    left, cs, right = cossin(np.asarray(u, dtype=complex), p=2, q=2)
    th = np.arctan2(np.diag(cs[2:, :2]), np.diag(cs[:2, :2]))  # C = cos th, S = sin th (per bit 0)

    def multiplexed(m):  # block_diag(a, b) over bit 1, acting on qubit 0
        a, b = m[:2, :2], m[2:, 2:]
        t, p, l, _ = u3_params(a)
        t2, p2, l2, al2 = u3_params(b @ a.conj().T)
        return [("u3", (t, p, l), (0,)), ("u1", (al2,), (1,)), ("cu3", (t2, p2, l2), (1, 0))]

    return (multiplexed(right) + [("ry", (2 * th[0],), (1,)), ("cry", (2 * (th[1] - th[0]),), (0, 1))]
            + multiplexed(left))


def _qasm_pieces(op, qs):
    """(name, params, qubits) pieces of one instruction in qelib1 gates: standard gates as they
    are, any other 1- or 2-qubit gate unrolled through its matrix (the reference unrolls the
    target to basis gates first, approximate_compiler.py:195, so its dumps never meets one)."""
    if op.name in _QASM_NAMES:
        return [(op.name, tuple(float(p) for p in op.params), qs)]
    if len(qs) == 1:
        t, p, l, _ = u3_params(op_matrix(op))
        return [("u3", (t, p, l), qs)]
    if len(qs) == 2:
        return [(nm, ps, tuple(qs[i] for i in loc)) for nm, ps, loc in unroll_two_qubit(op_matrix(op))]
    raise ValueError(f"qasm2_dumps: gate {op.name} on {len(qs)} qubits has no OpenQASM 2 form here")


def qasm2_dumps(circuit) -> str:
    """OpenQASM 2.0 text of a circuit (``qiskit.qasm2.dumps``; adapt_compiler.py:359-366 keeps
    one per layer in ``circuit_history``).  Gates outside qelib1 are unrolled (_qasm_pieces)."""
    lines = ["OPENQASM 2.0;", 'include "qelib1.inc";', f"qreg q[{circuit.num_qubits}];"]
    for ins in circuit.data:
        op = ins.operation
        if op.name in ("barrier", "delay"):
            continue
        for name, params, qs in _qasm_pieces(op, qubit_indices(circuit, ins)):
            ps = "(" + ",".join(repr(float(p)) for p in params) + ")" if params else ""
            lines.append(f"{name}{ps} " + ",".join(f"q[{q}]" for q in qs) + ";")
    return "\n".join(lines) + "\n"
