"""CPU oracle for the MPC/CEM planning hot path -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Importable only by `tests/`, `__graft_entry__.smoke()` and `bench.py` (cpu_baseline and parity
legs), and only as the checker. Parity pinning: golden vectors produced by running the reference's
own planner/model/cost code (`tests/golden/make_golden.py`), see oracle/cem.py's header.
"""
