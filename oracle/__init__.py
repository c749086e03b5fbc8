"""CPU oracle package — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker.  The product (blenderraytracer_amd, librt_hip.so) never imports or links anything here.
"""
