"""The reference-style testing driver (python -m dplasma_amd.testing), on CPU ranks."""
import os
import subprocess
import sys

import pytest

from helpers import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, nproc=1):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    if nproc == 1:
        cmd = [sys.executable, "-m", "dplasma_amd.testing", *args, "-g", "0"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m", "dplasma_amd.testing",
               *args, "-g", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    return r


@pytest.mark.parametrize("args", [
    "dpotrf -N 378 -t 93 -x", "zposv -N 150 -t 40 -K 3 -x", "sgemm -M 106 -N 283 -K 97 -t 56 -x",
    "dgeqrf -M 487 -N 283 -t 56 -i 8 -x", "dgeqrf_hqr -M 300 -N 200 -t 50 -i 10 --qr_a 2 -x",
    "dgetrf_incpiv -N 200 -t 50 -i 10 -x", "dgetrf_ptgpanel -N 200 -t 50 -x", "dlange -M 87 -N 83 -t 16 -x",
    # the remaining common.c flags: LAPACK storage (-A lld), cores, scheduler name, recursive hint, sync
    "dpotrf -N 300 -t 64 -A 320 -c 2 -o LFQ -z 32 -b -x", "dgemm -M 90 -N 70 -K 50 -t 16 -A 100 -B 60 -C 100 -x",
    # DTD drivers (testing_zpotrf_dtd, testing_zpotrf_dtd_untied, testing_zgemm_dtd)
    "dpotrf -N 300 -t 32 -o LL -x", "dgetrf_1d -N 200 -t 32 -o RND -x", "dgeqrf -M 300 -N 200 -t 40 -i 8 -o IP -x",
    "dpotrf_dtd -N 200 -t 32 -x", "dpotrf_dtd_untied -N 200 -t 32 -x", "dgemm_dtd -M 90 -N 70 -K 50 -t 16 -x",
    # DTD QR / incpiv LU, recursive QR (testing_zgeqrf_dtd[_untied], testing_zgetrf_incpiv_dtd, testing_zgeqrf_rd)
    "dgeqrf_dtd -M 150 -N 118 -t 32 -i 8 -x", "zgeqrf_dtd_untied -M 120 -N 90 -t 32 -i 8 -x",
    "dgetrf_incpiv_dtd -N 150 -t 32 -i 8 -x", "dgeqrf_rd -M 200 -N 150 -t 50 -i 10 -z 25 -x",
    # level-3 BLAS vs a dense reference, inverses
    "zhemm -M 90 -N 70 -t 16 -x", "dsymm -M 90 -N 70 -t 16 -u U -x", "zherk -N 90 -K 50 -t 16 -u U -x",
    "ssyrk -N 70 -K 40 -t 16 -x", "zher2k -N 90 -K 50 -t 16 -x", "dsyr2k -N 90 -K 50 -t 16 -u U -x",
    "dgeadd -M 90 -N 70 -t 16 -x", "ztrtri -N 150 -t 32 -u U -x", "dpoinv -N 150 -t 32 -x",
    # Q applications (all four side / trans combinations against the explicit Q)
    "dunmqr -M 120 -N 90 -K 40 -t 24 -i 8 -x", "zunmlq -M 90 -N 120 -K 40 -t 24 -i 8 -x",
    "dunmqr_hqr -M 150 -N 90 -K 30 -t 24 -i 8 --qr_a 2 -x", "dunmlq_systolic -M 90 -N 150 -K 30 -t 24 -i 8 -x",
    # solvers, reductions, QR tree validation
    "dgesv_incpiv -N 150 -t 32 -i 8 -K 3 -x", "dgesvd -M 150 -N 120 -t 24 -x", "zhbrdt -N 60 -t 6 -x",
    "dpivgen -M 400 -N 200 -t 20",
    # PTG -> DTD re-execution of the tile-DAG algorithms (the reference's --mca mca_pins ptg_to_dtd)
    "dgetrf_incpiv -N 150 -t 32 -i 8 -x --ptg-to-dtd", "zgelqf -M 100 -N 150 -t 25 -i 5 -x --ptg-to-dtd",
    # several runs: the operands are restored before every run (the reference re-generates them)
    "dpotrf -N 300 -t 64 -x --nruns 3", "dgetrf_1d -N 200 -t 32 -x --nruns 2", "dgeqrf -M 150 -N 100 -t 32 -i 8 -x --nruns 2",
])
def test_cli_single(args):
    r = _run(args.split())
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "[****] TIME(s)" in r.stdout and "SUSPICIOUS" not in r.stdout


def test_cli_multirank():
    r = _run("dgetrf_ptgpanel -N 200 -t 32 -P 2 -x".split(), nproc=4)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "PxQxg=   2 2" in r.stdout and "CORRECT" in r.stdout


def test_cli_unmqr_hqr_multirank():
    """Q application with an HQR tree on a 2 x 1 grid (testing_zunmqr_hqr with -P 2)."""
    r = _run("dunmqr_hqr -M 160 -N 96 -K 40 -t 16 -i 8 -P 2 --qr_a 2 -x".split(), nproc=2)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "CORRECT" in r.stdout and "SUSPICIOUS" not in r.stdout


def test_cli_kcyclic_multirank():
    """k-cyclic distribution (-s/-S: KP x KQ repetition) on a 2 x 2 grid."""
    r = _run("dpotrf -N 256 -t 32 -P 2 -s 2 -S 2 -x".split(), nproc=4)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "CORRECT" in r.stdout and "SUSPICIOUS" not in r.stdout


def test_cli_simulation_date():
    """--sim prints the critical path of tile-DAG algorithms with the reference SIMCOST weights
    (the reference prints parsec_getsimulationdate in simulation builds)."""
    env_args = ["dgeqrf", "-M", "64", "-N", "64", "-t", "32", "-i", "8", "--sim"]
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT, DPLASMA_QR_ENGINE="tile")
    r = subprocess.run([sys.executable, "-m", "dplasma_amd.testing", *env_args, "-g", "0"], capture_output=True,
                       text=True, timeout=600, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr
    assert "dgeqrf simulation M= 64 N= 64 NB= 32 : 26.0" in r.stdout, r.stdout
