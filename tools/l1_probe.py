"""Probe (timing only): the planned expansion's stream with a big net of L1 = 1024 (a 46 MB
table, 2.9 MB of rows per king-bucket pair) against L1 = 3072 (138 MB, 8.6 MB): does a row set
that fits an XCD's 4 MB L2 raise the hit rate?  The bench's games, chain 81, 3 steps."""
import json
import sys

sys.path.insert(0, ".")
from fishnet_amd import gpu_nnue as G, synthnet  # noqa: E402


def main():
    l1 = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    games, plies = 49152, 80
    nn = G.GpuNnue(synthnet.cached_synth_net(l1, 1), synthnet.cached_synth_net(128, 2))
    n = games * (plies + 1)
    d_p = nn.alloc(n * 32)
    nn.random_games_device(0x5EED0000, 0, games, plies, d_p)
    nn.synchronize()
    nn.time_expand_device(d_p, n, 1, 1)
    ms, t, st, rows = nn.time_expand_device(d_p, n, 1, 3)
    stream = nn.get_option(G.STAT_STREAM_NS) / 1e6
    print(json.dumps(dict(l1=l1, ms=ms / 3, stream=stream, plan=nn.get_option(G.STAT_PLAN_NS) / 1e6, rows=rows,
                          row_bytes=2 * l1 + 4, row_TBps=rows * (2 * l1 + 4) / stream / 1e9)), flush=True)


if __name__ == "__main__":
    main()
