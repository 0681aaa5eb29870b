"""Time the reference's own apf_step2 loop against the oracle's NumPy restatement, one
core, on the same frame (this container: the reference cannot travel to the GPU box).

    /opt/conda/bin/python3.9 tests/golden/time_reference.py [n] [nsrc] [accept_min] [--json F]

Runs apf_step2.py's loop lines (:298-338, or 3body :324-373) through the fixture
harness of tests/golden/make_golden.py (the reference's own function definitions and
setup, astropy 4.3.1 models, a stand-in comm) with burn_in past the run, so no chain
rows are stacked or written -- the sampling alone -- and then oracle/olpe_oracle.py's
Walker over the same number of iterations.  Prints iterations per second of each; with ``--json F`` also merges them into F
(profiles/r04/reference_cpu_timing.json, keyed "<n>x<n>_<nsrc>", with the CPU model), the
file bench.py reads for ``cpu_baseline.reference_over_port``.
(Test infrastructure, like bench.py's cpu_baseline leg: the oracle is timed as the CPU
baseline, never as the product.)
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import make_golden as mg  # noqa: E402  (needs astropy 4.3.1: /opt/conda/bin/python3.9)
from olpefit_amd import synth  # noqa: E402
from oracle import olpe_oracle as ora  # noqa: E402


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def main():
    argv = list(sys.argv[1:])
    out = None
    if "--json" in argv:
        i = argv.index("--json")
        out = argv[i + 1]
        del argv[i:i + 2]
    n = int(argv[0]) if len(argv) > 0 else 64
    nsrc = int(argv[1]) if len(argv) > 1 else 2
    accept_min = int(argv[2]) if len(argv) > 2 else 60
    spec = mg.TWO if nsrc == 2 else mg.THREE
    image, _ = synth.make_image(n, nsrc, seed=0)
    image = image.astype(">f4")
    header = dict((k.lower(), v) for k, v in synth.HEADER.items())
    guess = synth.guess_values(n, nsrc)
    t0 = time.perf_counter()
    trace, p0, _ = mg.run_reference_loop(spec, image, header, guess, 1000, accept_min,
                                          10 ** 9, "/tmp", 0)
    t_ref = time.perf_counter() - t0
    iters = len(trace)
    dm, err, _, _ = ora.noise_model(np.asarray(image, dtype=np.float32), 1.0, 1, 1, 2)
    t0 = time.perf_counter()
    ora.Walker(dm, err, p0, 1000, nsrc=nsrc).run(iters, burn_in=10 ** 9)
    t_ora = time.perf_counter() - t0
    print(f"{n}x{n}, {nsrc} sources, {iters} iterations, one core:")
    print(f"  reference apf_step2 loop (astropy 4.3.1): {iters / t_ref:9.1f} iterations/s "
          f"({t_ref / iters * 1e3:.3f} ms per iteration)")
    print(f"  oracle NumPy restatement (bench.py cpu_baseline): {iters / t_ora:9.1f} iterations/s "
          f"({t_ora / iters * 1e3:.3f} ms per iteration)")
    if out:
        import json
        try:
            with open(out) as f:
                data = json.load(f)
        except (OSError, ValueError):
            data = {}
        data[f"{n}x{n}_{nsrc}"] = {
            "image": f"{n}x{n}", "sources": nsrc, "iterations": iters,
            "reference_iters_per_s": iters / t_ref, "port_iters_per_s": iters / t_ora,
            "reference_over_port": t_ora / t_ref, "port_over_reference": t_ref / t_ora,
            "cores": 1, "cpu_model": cpu_model(),
            "reference": "apf_step2.py loop lines :298-338 (3body :324-373) with astropy "
                         "4.3.1, run by tests/golden/make_golden.py's harness",
            "port": "oracle/olpe_oracle.py Walker (bench.py's cpu_baseline)"}
        with open(out, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
