"""CPU oracle for parity tests and the cpu_baseline leg of bench.py — TEST INFRASTRUCTURE.

Nothing under itrails_amd/ imports this package; only tests/, __graft_entry__.smoke() and
bench.py (cpu_baseline) do, and only as the checker, never as the thing measured or shipped.
"""
