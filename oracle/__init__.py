"""CPU oracle (test infrastructure only): restatements of the reference algorithms.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import this
package; the product package never does.
"""
