"""The reference's node graph as a host-side pipeline: scanRegistration -> laserOdometry ->
laserMapping, each node on its own engine context (own HIP stream, own device state) and its own
thread, connected by FIFO queues that play the ROS topics.

The reference runs the four nodes as separate processes ("odometry and mapping
running in parallel", reference README.md:42): while laserMapping solves frame k, laserOdometry is
already on frame k+1 and scanRegistration on frame k+2.  Each node consumes its own topic in order,
so every node sees exactly the inputs it sees in a sequential run and the outputs are identical;
only the overlap changes.  The engine calls release the GIL (ctypes), so the three threads' host
copies and the three contexts' kernels overlap on the device.

Topics (reference file:line of the publish / subscribe pair):
  features   /laser_cloud_sharp .. /velodyne_cloud_2   scanRegistration.cpp:593-635 -> laserOdometry.cpp:365-379
  odometry   /laser_cloud_corner_last, _surf_last, /velodyne_cloud_3, /laser_odom_to_init
             laserOdometry.cpp:858-930 -> laserMapping.cpp:353-366
Mapping consumes a frame only when odometry published it (every skipFrameNum-th frame, `pub == 7`).
"""
import queue
import threading
import time

_END = object()


class NodePipeline:
    """Three node contexts on three threads.  `engine_cls(cfg)` makes one context; `imu` entries are
    not routed here (configs 3/4 carry none; the IMU path is the single-context `Engine.imu`)."""

    # measured on config 3 (tools/pipe_bench.py, GPU_MAX_HW_QUEUES=8): laserMapping is the critical
    # node; its streams at the highest priority take the pipeline from 0.63-0.71 to 0.60-0.62 ms/sweep
    DEFAULT_PRIORITY = {"mp": 1}

    def __init__(self, engine_cls, cfg=None, depth=4, stages=3, priority=DEFAULT_PRIORITY):
        """stages = 3: one context / thread per node; 2: scanRegistration and laserOdometry share
        one context and thread (the front end), laserMapping has its own.  priority: optional
        {"sr" | "od" | "mp": > 0 high, 0 normal, < 0 low} stream priorities of the node contexts."""
        if stages not in (2, 3):
            raise ValueError("stages must be 2 or 3")
        # each node context drops the batch pipeline's extra streams before the next is made, so that
        # the contexts' streams spread over the process's hardware queues (0.59 -> 0.46 ms/sweep)
        def node():
            e = engine_cls(cfg)
            if hasattr(e, "set_tuning"):
                e.set_tuning(batch_streams=0)
            return e
        self.sr = node()
        self.od = node() if stages == 3 else self.sr
        self.mp = node()
        self.stages = stages
        self.depth = depth
        for k, v in (priority or {}).items():
            getattr(self, k).set_stream_priority(v)

    def close(self):
        for e in {id(e): e for e in (self.sr, self.od, self.mp)}.values():
            e.close()

    def run(self, sweeps, stamps=None, on_mapping=None):
        """feed `sweeps` (raw (n, >=3) float32 clouds) in order; returns (mapping results in frame
        order as (aft, bef, registered) tuples, number of sweeps odometry processed).  Raises the
        first node error after all threads have stopped."""
        q_feat = queue.Queue(self.depth)
        q_odom = queue.Queue(self.depth)
        results, err = [], []
        n_od = [0]
        busy = {"scanRegistration": 0.0, "laserOdometry": 0.0, "laserMapping": 0.0}

        def guard(fn, out_q):
            def body():
                try:
                    fn()
                except BaseException as e:  # noqa: BLE001 - re-raised in the caller
                    err.append(e)
                finally:
                    if out_q is not None:
                        out_q.put(_END)
            return body

        def node_sr():
            for k, s in enumerate(sweeps):
                if err:
                    return
                t = stamps[k] if stamps is not None else 0.1 * k
                a = time.perf_counter()
                rc, f = self.sr.scan_registration(s, stamp=t)
                busy["scanRegistration"] += time.perf_counter() - a
                if rc == 0:
                    if self.stages == 3:
                        q_feat.put((t, f))
                    else:
                        odometry(t, f)

        def odometry(t, f):
            n_od[0] += 1
            a = time.perf_counter()
            pub, pose, cl, sl, full = self.od.odometry(f, stamp=t)
            busy["laserOdometry"] += time.perf_counter() - a
            if pub == 7:
                q_odom.put((t, pose, cl, sl, full))

        def node_od():
            while True:
                it = q_feat.get()
                if it is _END:
                    return
                if err:
                    continue  # drain so the producer never blocks
                try:
                    odometry(*it)
                except BaseException as e:  # noqa: BLE001 - keep draining, re-raised in the caller
                    err.append(e)

        def node_mp():
            while True:
                it = q_odom.get()
                if it is _END:
                    return
                if err:
                    continue
                t, pose, cl, sl, full = it
                try:
                    a = time.perf_counter()
                    r = self.mp.mapping(pose, cl, sl, full, stamp=t)
                    busy["laserMapping"] += time.perf_counter() - a
                    results.append(r)
                    if on_mapping is not None:
                        on_mapping(self.mp, r)
                except BaseException as e:  # noqa: BLE001 - keep draining, re-raised in the caller
                    err.append(e)

        if self.stages == 3:
            threads = [threading.Thread(target=guard(node_sr, q_feat), name="scanRegistration"),
                       threading.Thread(target=guard(node_od, q_odom), name="laserOdometry")]
        else:
            threads = [threading.Thread(target=guard(node_sr, q_odom), name="frontEnd")]
        threads.append(threading.Thread(target=guard(node_mp, None), name="laserMapping"))
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        self.busy_s = busy  # seconds each node spent inside its engine calls (the rest is waiting)
        if err:
            raise err[0]
        return results, n_od[0]
