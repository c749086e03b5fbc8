"""Ownership of the LDS pool launches' work queues (blenderraytracer_amd/csrc/queue_slots.h): the CPU
test of the allocator that replaced round 5's 1024-slot ring.

tests/hostcheck/queue_slots_check.cpp runs simulated launches on many threads — acquire, hold with a
release token, end (ownership cleared before the token completes), cancels that extend the release to a
later token, failed enqueues that abandon the slot — and counts every slot handed out while another
launch still owned it.  The GPU side (a long render + 2048 small LDS-pool launches in flight) is
tests/test_gpu_parity.py::test_lds_queues_owned_under_concurrent_launches.
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "hostcheck", "queue_slots_check.cpp")
HDR = os.path.join(ROOT, "blenderraytracer_amd", "csrc", "queue_slots.h")
BIN = os.path.join(HERE, "hostcheck", "_build", "queue_slots_check")


@pytest.fixture(scope="module")
def checker():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    if not os.path.exists(BIN) or any(os.path.getmtime(BIN) < os.path.getmtime(p) for p in (SRC, HDR)):
        tmp = "%s.tmp%d" % (BIN, os.getpid())    # parallel test workers: build aside, rename atomically
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-Wall", SRC, "-o", tmp])
        os.replace(tmp, BIN)
    return BIN


def run(binary, threads, launches, slots, broken):
    out = subprocess.run([binary, str(threads), str(launches), str(slots), str(int(broken))],
                         capture_output=True, text=True, timeout=120, check=True).stdout
    return {k: int(v) for k, v in re.findall(r"(\w+)=(\d+)", out)}


@pytest.mark.parametrize("slots", [4, 16, 1024])
def test_no_slot_handed_out_twice_while_held(checker, slots):
    r = run(checker, 8, 20000, slots, False)
    assert r["violations"] == 0, r
    assert r["acquired"] == 8 * 20000
    assert r["extended"] > 1000 and r["abandoned"] > 1000
    if slots == 4:
        assert r["waits"] > 0        # the threads really ran out of slots and waited


def test_checker_catches_a_ring_without_ownership(checker):
    """Mutation: a completion test that always says "done" (round 5's ring) is caught."""
    r = run(checker, 8, 5000, 4, True)     # 4 slots: one thread alone holds up to 7 launches
    assert r["violations"] > 0, r
