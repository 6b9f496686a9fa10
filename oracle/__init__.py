"""CPU oracle of the POMS hot path -- TEST INFRASTRUCTURE ONLY.

May be imported only by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``, as the checker / baseline.  The product
package ``poms_amd`` never imports it.
"""
