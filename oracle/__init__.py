"""Oracle: CPU restatements of the reference rollout (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / CPU baseline. Parity status: *parity unpinned* (the reference has
no tests or fixtures for this path and its Python may not be executed here).
"""
