"""Re-run the first STEPS steps of a parity fixture's reference side (tests/golden/make_parity_train.py,
needs /root/reference; CPU) at a given torch thread count and report the first step whose batch loss
differs from the committed fixture.  Round 5 used it to explain ADVICE r4's "s6/s7 PSNR moved": with
ONE thread seeds 0, 6 and 7 reproduce their fixtures bit for bit over 200 steps; with 8 threads the
losses part at step 10-12 (the CPU reductions' order follows the thread count).

    python tools/parity_fixture_check.py SEED THREADS [STEPS=200]
"""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    seed, threads = int(sys.argv[1]), int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    # one short epoch at the schedule's first rate (= the first STEPS steps of the 10-epoch protocol)
    os.environ.update(MFNERF_PARITY_EPOCHS="1", MFNERF_PARITY_EPOCH_STEPS=str(steps), MFNERF_PARITY_TEST_VIEWS="1",
                      MFNERF_PARITY_THREADS=str(threads))
    sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests"), ROOT,
                    os.path.join(ROOT, "mf-nerf_amd")]
    import make_parity_train as M
    name = "parity_train.json" if seed == 0 else f"parity_train_s{seed}.json"
    fixture = json.load(open(os.path.join(ROOT, "tests", "golden", name)))["loss_every_step"][:steps]
    with tempfile.TemporaryDirectory() as d:
        M.HERE = d  # the re-run's JSON goes here, not over the fixture
        M.main(seed)
        got = json.load(open(os.path.join(d, name)))["loss_every_step"]
    first = next((i + 1 for i, (a, b) in enumerate(zip(got, fixture)) if a != b), None)
    print(json.dumps({"seed": seed, "threads": threads, "steps": steps, "first_differing_step": first,
                      "ratio_at_last": got[-1] / fixture[-1]}))


if __name__ == "__main__":
    main()
