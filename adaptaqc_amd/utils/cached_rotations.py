# (C) Copyright IBM 2025.
#
# This code is licensed under the Apache License, Version 2.0. You may
# obtain a copy of this license in the LICENSE.txt file in the root directory
# of this source tree or at http://www.apache.org/licenses/LICENSE-2.0.
#
# Any modifications or derivative works of this code must retain this
# copyright notice, and modified files need to carry a notice indicating
# that they have been altered from the originals.
#
# Modified for adaptaqc_amd: this file restates the reference file named in its docstring
# (qiskit-community/adapt-aqc) on top of the MI355X engine (libaqchip); it has been altered
# from the original.

"""Cached, batched Rotoselect / Rotosolve evaluation.

The reference (cost_minimiser.py:267-368) re-simulates the whole circuit for every candidate of
every rotation gate: 3 evaluations per gate for Rotosolve, 1 + 3 x 2 = 7 for Rotoselect.  The
candidates differ in one single-qubit gate, so:

* Statevector, global cost: with phi = P|0> (gates before the one being varied, already
  updated) and chi = S^dag|0> (gates after it, undone), every candidate's amplitude is
  <0|S V P|0> = sum_ab V[a][b] T[a][b] with T = aqc_sv_transition(chi, phi, q).  Moving to the
  next gate applies the (new) current gate to phi and the next (old) gate to chi, so a whole
  sweep costs about three circuit simulations instead of 3-7 per gate.  Costs are exact: the
  same numbers the reference's simulations produce, up to rounding.
* MPS, global cost: truncation makes chi = S^dag|0> differ from the forward replay the
  reference does, so only the prefix is cached (the MPS after the gates before the varied
  one, which is what every replay computes first) and the candidates replay the suffix together
  in lock-step batched launches (aqc_mps_copy_batch / apply_batch), then <0|psi> of each through
  the sites it rewrote against rows cached on the prefix (aqc_mps_zero_hw1_batch).
* MPS, local cost (0.5 (1 - mean <Z_i>), aer_mps_backend.py:72-74, 80-86) or softened global cost
  (1 - |<0|psi>|^2 - alpha sum_i |<e_i|psi>|^2, :49-70): the same prefix batch, then every
  candidate's sum of <Z_i> (aqc_mps_z_sum_batch: a candidate differs from the prefix only on the
  sites its gate, the suffix and the sort rewrote, so it contracts those against environments of
  sum_i Z_i cached on the prefix) or HW-1 amplitudes (aqc_mps_zero_hw1_batch, the same window
  against the prefix's Hamming-weight-1 rows) in one set of launches.
* Statevector, local cost (aer_sv_backend.py:32-35, 49-59): no transition shortcut (every <Z_i> of
  every candidate); the prefix state is cached and the candidates replay the suffix from it.
  The softened cost raises on the statevector backend, as in the reference (generic path).

The compiler's ``cost_evaluation_counter`` advances by the number of evaluations the reference
would have made, so histories and logs stay comparable.
"""
import numpy as np

from .. import gates as G
from .._lib import OP_DTYPE, ops_array
from ..circuit import device_ops, device_ops_rows
from ..device import DeviceSV, apply_batch, check_batch, copy_batch, z_sum_batch, zero_hw1_batch


class _View:
    """``circuit.data[lo:hi]`` with the circuit's own qubit resolution: this IR's circuits or the
    reference's qiskit circuits (``find_bit``), so the evaluators also serve the reference's own
    CostMinimiser under reference_binding.install()."""

    def __init__(self, circuit, lo, hi):
        self.data = circuit.data[lo:hi]
        self.num_qubits = circuit.num_qubits
        self._c = circuit

    def find_bit(self, q):
        return self._c.find_bit(q)


def _ops(circuit, lo, hi):
    return device_ops(_View(circuit, lo, hi))


def _inverse_ops(ops):
    return [(np.conj(np.asarray(m)).T, qs) for m, qs in reversed(ops)]


def _ops_qubit(circuit, index):
    """Integer qubit of the single-qubit gate at ``index`` (this IR or qiskit-shaped)."""
    from ..circuit import qubit_indices

    return qubit_indices(circuit, circuit.data[index])[0]


class _SweepBase:
    def __init__(self, compiler):
        self.compiler = compiler
        self.pos = None

    def count(self, k):
        self.compiler.cost_evaluation_counter += k


class SVTransitionSweep(_SweepBase):
    """Exact costs of all single-qubit candidates at one position from a 2x2 transition matrix."""

    def __init__(self, compiler):
        super().__init__(compiler)
        n = compiler.full_circuit.num_qubits
        self.phi = DeviceSV(n)
        self.chi = DeviceSV(n)

    def goto(self, index):
        circ = self.compiler.full_circuit
        if self.pos is None or index < self.pos:
            self.phi.reset()
            self.phi.apply(_ops(circ, 0, index))
            self.chi.reset()
            self.chi.apply(_inverse_ops(_ops(circ, index + 1, len(circ.data))))
        elif index > self.pos:
            self.phi.apply(_ops(circ, self.pos, index))
            self.chi.apply(_ops(circ, self.pos + 1, index + 1))
        self.pos = index

    def costs(self, index, mats):
        circ = self.compiler.full_circuit
        q = _ops_qubit(circ, index)
        t = self.chi.transition(self.phi, q)
        return [float(1.0 - abs(np.sum(m * t)) ** 2) for m in mats]


def _cost_kind(compiler):
    if getattr(compiler, "optimise_local_cost", False):
        return "local"
    if getattr(compiler, "soften_global_cost", False):
        return "soft"
    return "global"


def _soften_alpha(compiler):
    """aer_mps_backend.py:63-66: alpha = |C_prev - sufficient_cost|, C_prev the last global cost of
    the history (1 when empty) -- read per evaluation, as the reference does."""
    hist = compiler.global_cost_history
    previous_cost = hist[-1] if len(hist) > 0 else 1
    return abs(previous_cost - compiler.adapt_config.sufficient_cost)


class MPSPrefixBatch(_SweepBase):
    """Prefix MPS cached across candidates and gates; candidates replay the suffix in one batch,
    then the compiler's cost (global, softened global or local) of every candidate together."""

    def __init__(self, compiler, kind="global"):
        super().__init__(compiler)
        self.backend = compiler.backend
        self.phi = None
        self.kind = kind
        # (instruction ids, rows of the whole circuit, row offsets, first row, the instructions --
        # held so that no id in the key can be reused by a new instruction while it is cached)
        self._conv = None

    def _rows(self, circ, lo, hi):
        """device_ops_rows(circ, lo, hi) from one conversion per circuit state: a gate's visit asks
        for the prefix advance (goto) and the suffix (costs) of the same circuit, and each call of
        the memoised conversion still walks every instruction in Python (~0.15 ms at 150 gates).
        The conversion is reused while no instruction object was replaced (replace_1q_gate swaps
        the instruction; an in-place parameter change would go unnoticed, which no caller of the
        cached evaluator makes between a goto and its costs)."""
        data = circ.data
        ids = tuple(map(id, data))
        if self._conv is not None and self._conv[0] != ids and len(self._conv[0]) == len(ids):
            self._patch(circ, ids)
        if self._conv is None or self._conv[0] != ids:
            start = 1 if len(data) and data[0].operation.name == "set_matrix_product_state" else 0
            full = device_ops_rows(circ, start, len(data))
            from ..circuit import _memo_get

            prev = _memo_get(circ)
            if prev is None or prev[0] != start:
                return device_ops_rows(circ, lo, hi)
            size = OP_DTYPE.itemsize
            off = np.cumsum([0] + [len(e[3]) // size for e in prev[1]])
            self._conv = (ids, full, off, start, tuple(data))
        _, full, off, start, _ = self._conv
        lo, hi = max(lo, start), min(hi, len(data))
        if hi <= lo:
            return full[:0]
        return full[off[lo - start]:off[hi - start]]

    def _patch(self, circ, ids):
        """The sweep replaced a few instructions since the last conversion (the visited gate):
        re-convert just those into the cached rows when each keeps its row count, else drop the
        cache (the next _rows converts the circuit again)."""
        from ..circuit import _Range

        old_ids, full, off, start, _ = self._conv
        changed = [i for i, (a, b) in enumerate(zip(ids, old_ids)) if a != b]
        if not changed or len(changed) > 4 or changed[0] < start:
            self._conv = None
            return
        for i in changed:
            rows = ops_array(device_ops(_Range(circ, i, i + 1)))
            a, b = off[i - start], off[i - start + 1]
            if len(rows) != b - a:
                self._conv = None
                return
            full[a:b] = rows
        self._conv = (ids, full, off, start, tuple(circ.data))

    def _grown(self, e):
        """A capacity overflow of an unbounded run: the backend grew its capacity, so the prefix
        is rebuilt at the new one (the retry replays it)."""
        if not self.backend.grow_on_overflow(e):
            return False
        self.phi, self.pos = None, None
        return True

    def goto(self, index):
        while True:
            try:
                return self._goto(index)
            except Exception as e:
                if not self._grown(e):
                    raise

    def costs(self, index, mats):
        while True:
            try:
                return self._costs(index, mats)
            except Exception as e:
                if not self._grown(e):
                    raise
                self.goto(index)

    def _goto(self, index):
        circ = self.compiler.full_circuit
        base, start = self.backend.ensure_base(circ)
        if self.phi is None or self.phi.chi_cap != base.chi_cap:
            self.phi, self.pos = self.backend.new_state(), None
        # the prefix's advance is queued (aqc_mps_apply_batch_async); its error flags are read with
        # the candidates' after their costs (costs() always follows goto()), so a gate costs one
        # host wait instead of three
        if self.pos is None or index < self.pos:
            self.phi.copy_from(base)
            self._advance(self._rows(circ, start, index))
        elif index > self.pos:
            self._advance(self._rows(circ, self.pos, index))
        self.pos = index

    def _advance(self, rows):
        if len(rows):
            apply_batch([self.phi], [rows], wait=False)

    def _costs(self, index, mats):
        circ = self.compiler.full_circuit
        q = _ops_qubit(circ, index)
        # the suffix's rows from the circuit's memoised conversion (device_ops_rows), the candidates'
        # gates in one conversion, each list joined as bytes (a structured-array concatenate costs
        # ~16 us)
        suffix = self._rows(circ, index + 1, len(circ.data)).tobytes()
        cand = ops_array([(m, (q,)) for m in mats]).tobytes()
        size = len(cand) // len(mats)
        states = self.backend.scratch_states(len(mats))
        copy_batch(states, [self.phi] * len(mats))
        lists = [np.frombuffer(cand[i * size:(i + 1) * size] + suffix, dtype=OP_DTYPE) for i in range(len(mats))]
        # queued; the prefix's and the candidates' error flags are read after the costs' read-back
        apply_batch(states, lists, sort=True, wait=False)
        if self.kind == "local":
            # only sum_i <Z_i> enters the cost: each candidate contracts the sites it rewrote
            # against the prefix's cached environments (aqc_mps_z_sum_batch)
            n = circ.num_qubits
            zs = z_sum_batch(self.phi, states)
            check_batch([self.phi] + states)
            return [float(0.5 * (1 - t / n)) for t in zs]
        # <0|psi> (and the softened cost's <e_i|psi>) likewise through the rewritten sites against
        # rows cached on the prefix (aqc_mps_zero_hw1_batch)
        # (its read-back also carries the prefix's and the candidates' error flags)
        ov, amps = zero_hw1_batch(self.phi, states, amps=self.kind == "soft")
        costs = [float(1.0 - abs(v) ** 2) for v in ov]
        if self.kind == "soft":
            alpha = _soften_alpha(self.compiler)
            costs = [c - alpha * float(np.sum(np.abs(a) ** 2)) for c, a in zip(costs, amps)]
        return costs


class SVPrefixBatch(_SweepBase):
    """Statevector, local cost: the prefix state cached across candidates and gates (advanced gate
    by gate as the sweep moves); each candidate replays its gate and the suffix from it, then
    <Z_i> of every qubit (aqc_sv_z_all)."""

    def __init__(self, compiler):
        super().__init__(compiler)
        n = compiler.full_circuit.num_qubits
        self.phi = DeviceSV(n)
        self.cand = []

    def goto(self, index):
        circ = self.compiler.full_circuit
        if self.pos is None or index < self.pos:
            self.phi.reset()
            self.phi.apply(_ops(circ, 0, index))
        elif index > self.pos:
            self.phi.apply(_ops(circ, self.pos, index))
        self.pos = index

    def costs(self, index, mats):
        circ = self.compiler.full_circuit
        q = _ops_qubit(circ, index)
        suffix = ops_array(_ops(circ, index + 1, len(circ.data)))
        while len(self.cand) < len(mats):
            self.cand.append(DeviceSV(self.phi.n))
        # every candidate's replay queued first (each state has its own stream, so the candidates'
        # passes run side by side: two or more tile workgroups per CU), the <Z_i> read afterwards
        for m, st in zip(mats, self.cand):
            st.copy_from(self.phi)
            st.apply(np.concatenate([ops_array([(m, (q,))]), suffix]))
        return [float(0.5 * (1 - np.mean(st.z_all()))) for st in self.cand[:len(mats)]]


def make_evaluator(compiler):
    """The cached evaluator for the compiler's current settings, or None (generic path)."""
    from ..backends.aer_mps_backend import AerMPSBackend
    from ..backends.aer_sv_backend import AerSVBackend

    kind = _cost_kind(compiler)
    if isinstance(compiler.backend, AerMPSBackend):
        return MPSPrefixBatch(compiler, kind)
    if isinstance(compiler.backend, AerSVBackend):
        if kind == "global":
            return SVTransitionSweep(compiler)
        if kind == "local":
            return SVPrefixBatch(compiler)
    return None  # (the softened cost on the statevector backend raises, as the reference does)


def rotation(name, theta):
    return G.one_qubit(name, [theta])
