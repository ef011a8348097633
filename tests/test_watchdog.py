"""Hang watchdog: a process that stops making progress aborts itself (so torchrun tears the group down)."""
import os
import subprocess
import sys
import textwrap

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _run(body, timeout=60):
    code = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        from photon_ml_amd.utils.watchdog import start_watchdog, EXIT_CODE
        from photon_ml_amd.utils.timing import trace_range
        {body}
    """)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)


def test_stalled_rank_aborts_with_stack_dump():
    r = _run("""
        start_watchdog(0.5)
        time.sleep(30)   # a stuck collective
        print("unreachable")
    """)
    assert r.returncode == 75, (r.returncode, r.stderr[-2000:])
    assert "no progress" in r.stderr and "time.sleep" not in r.stdout
    assert "File" in r.stderr  # faulthandler stack of the stuck thread


def test_heartbeats_keep_a_progressing_rank_alive():
    r = _run("""
        start_watchdog(0.6)
        for _ in range(20):          # 2 s of work, well past the timeout, with a heartbeat every 0.1 s
            with trace_range("step"):
                time.sleep(0.1)
        print("done")
    """)
    assert r.returncode == 0 and "done" in r.stdout, r.stderr[-2000:]
