"""CPU: the oracle and the host emulator of the product pipeline (its kernel bodies and orchestration) built
into one executable with -fsanitize=address,undefined (tests/sanitize) and run on small fields,
partial / shuffled edge lists, lifting and Farneback — clean under the sanitizers and emulator == oracle."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.join(ROOT, "tests", "sanitize")


def test_oracle_and_emulator_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(HERE, "_build", "san_driver")], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "clean and equal" in r.stdout
