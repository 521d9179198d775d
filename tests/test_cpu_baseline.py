"""The reported CPU baseline pipeline computes what the reference computes."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_baseline_matches_oracle(oracle):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "baseline"])
    exe = os.path.join(ROOT, "oracle", "_build", "fc_cpu_baseline")
    out = subprocess.run([exe, "--verify"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert '"verify": true' in out.stdout
