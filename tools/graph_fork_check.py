"""Do forked branches of a captured HIP graph run concurrently on this ROCm?  Two small-grid kernels
(torch.cuda._sleep, one workgroup each) captured on one stream, then on two streams forked from the
capture stream and joined; replay time of each graph.  Concurrent branches replay in about half
the time of the serial graph."""
import json
import time

import torch


def timed(g, reps=50):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    dev = torch.device('cuda:0')
    side = torch.cuda.Stream(dev)
    out = {}
    for cyc, name in ((200000, 'serial'), (200000, 'forked'), (2000, 'serial_tiny'), (2000, 'forked_tiny')):
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            main_s = torch.cuda.current_stream(dev)
            if name.startswith('serial'):
                torch.cuda._sleep(cyc)
                torch.cuda._sleep(cyc)
            else:
                side.wait_stream(main_s)
                torch.cuda._sleep(cyc)
                with torch.cuda.stream(side):
                    torch.cuda._sleep(cyc)
                main_s.wait_stream(side)
        timed(g, 5)
        out[name + '_us'] = round(timed(g), 1)
    out['concurrent'] = out['forked_us'] < 0.75 * out['serial_us']
    out['fork_join_overhead_us'] = round(out['forked_tiny_us'] - out['serial_tiny_us'], 1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
