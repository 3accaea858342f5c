"""Host checks of integer identities the kernels rely on (no GPU needed).

render_kernel decodes a job q into (sample, pixel) and a pixel into (row,
column) by q / d = umulhi(2q, ceil(2^31 / d)) (rtmi_device.hip, camera_ray /
adopt): exact for every tile size d in 1..64 and every job index the host
allows (q < 64 * 65535 < 2^22, rtmi_device.hip's chunk clamp)."""
import numpy as np


def test_job_division_by_reciprocal_multiply_is_exact():
    q = np.arange(1 << 22, dtype=np.uint64)
    for d in range(1, 65):
        m = np.uint64(0x7FFFFFFF // d + 1)
        assert np.array_equal(((q << np.uint64(1)) * m) >> np.uint64(32), q // np.uint64(d)), d


def test_camera_ray_pool_assigns_the_same_jobs():
    """render_kernel's camera-ray pool, restated on the host:
    lane L of the pool holds job pbase + L; in a pass where the lanes in mask m
    finished, the lane of rank r among them takes slot ppos + r, refilling the
    pool (pbase += 64) when it runs out.  Every lane gets exactly the job the
    plain scheme gives it (next + rank, next += popcount(m)), so each
    (pixel, sample) keeps its ray and stream, and every job is taken once."""
    rng = np.random.default_rng(7)
    for nq in (1, 37, 64, 65, 500, 64 * 21):
        # plain scheme and pool scheme side by side
        job_plain = np.arange(64)
        job_pool = np.arange(64)
        active = job_plain < nq
        nxt, pbase, ppos = 64, 0, 64
        taken = [int(j) for j in job_plain[active]]
        while active.any():
            done = active & (rng.random(64) < 0.37)
            ranks = np.cumsum(done) - 1
            cnt = int(done.sum())
            for lane in np.flatnonzero(done):
                job_plain[lane] = nxt + ranks[lane]
            nxt += cnt
            served = 0
            while served < cnt:
                if ppos == 64:
                    pbase, ppos = pbase + 64, 0
                take = min(cnt - served, 64 - ppos)
                for lane in np.flatnonzero(done):
                    r = ranks[lane] - served
                    if 0 <= r < take:
                        job_pool[lane] = pbase + ppos + r
                ppos += take
                served += take
            assert np.array_equal(job_plain[done], job_pool[done])
            for lane in np.flatnonzero(done):
                if job_pool[lane] < nq:
                    taken.append(int(job_pool[lane]))
                else:
                    active[lane] = False
        assert sorted(taken) == list(range(nq)), nq
