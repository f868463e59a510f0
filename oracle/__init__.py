"""CPU parity oracle for the ADAPT-AQC overlap / gradient hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``adaptaqc_amd/`` imports this package;
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` use it, and only as the checker / baseline, never as the product.

The reference (qiskit-community/adapt-aqc) is pure Python whose arithmetic lives in
un-vendored third-party code that is absent from this image:

* qiskit-aer ~=0.16.0 (setup.py:18) -- statevector and matrix-product-state simulators;
* aqc_research.mps_operations (setup.py:25, git+ssh, un-pinned commit) -- MPS helpers;
* qiskit ~=1.3.1 (setup.py:17) -- circuit IR and gate matrices.

Importing the reference fails with an ordinary ``ModuleNotFoundError`` (not a
permission denial), so this package restates the published algorithms of those
dependencies in numpy, following the reference call sites cited in each function.
It is pinned by the reference's own known-answer tests and fixtures
(SURVEY.md section 8(c)); see ``tests/test_oracle_*.py``.  Aer's truncation details
when ``max_bond_dimension`` binds cannot be checked offline: results in that
regime are "parity unpinned" (DESIGN.md).
"""
