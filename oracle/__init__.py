"""CPU oracle for the swarm-RL hot path — TEST INFRASTRUCTURE ONLY.

Checker, never product: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` import this package.  See
``oracle/swarm_oracle.py`` for what is restated and where it is pinned.
"""
