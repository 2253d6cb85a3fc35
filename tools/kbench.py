"""Per-kernel timing of the CNN step kernels at several batch sizes (CUDA events)."""
import sys
import torch
sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
from pytorch_distributed_mnist_amd.runtime.program import build_local_program
from pytorch_distributed_mnist_amd.runtime.cnn_step import choose_bands, choose_ipb

train = synthetic_split(60000, True)
test = synthetic_split(512, False)


def timeit(fn, iters=50):
    """GPU time per call: `iters` back-to-back calls captured into one hipGraph and replayed
    (eager launches through the bindings would measure host overhead for small kernels)."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * iters) * 1e3



def main():
  for B in [int(b) for b in (sys.argv[1:] or ["256", "1024", "4096"])]:
      p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                              use_graphs=False)
      p.optimizer.sync_hyperparams()
      p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
      st = p.gpu
      C, P, G = st.C, st.P, st.G
      ldt = -(-B // 32) * 32
      S = st.splitk_train
      bands = choose_bands(B)
      ipb = choose_ipb(B) if bands == 1 else 1
      nblk = C.cnn_bwd_nblk(B, ipb, bands)
      st.train_step(B)
      torch.cuda.synchronize()
      z = torch.zeros(1, dtype=torch.int64, device="cuda")
      ks = {
          "cnn_fwd": lambda: C.cnn_fwd(st.ep_images.view(-1, 784), st.ep_labels, None, z, B, B,
                                       P["conv1.weight"], P["conv1.bias"], st.w2, P["conv2.bias"],
                                       st.pool, st.pmask, *st.fwd_outputs(B)),
          "fc1_fwd": lambda: C.fc1_fwd(st.pool, st.wf1, st.part, B, S),
          "cnn_head": lambda: C.cnn_head(st.part, S, B, P["fc1.bias"], P["fc2.weight"], P["fc2.bias"],
                                         st.ylab, True, st.dh, st.dht, ldt, st.head_slab,
                                         st.metrics.train_view(), None, None),
          "fc1_bwd": lambda: C.fc1_bwd(st.dh, st.dht, ldt, st.pool, st.current_wf1t(), B, G["fc1.weight"],
                                       st.dpool, st.head_slab, G["fc2.weight"], G["fc2.bias"],
                                       G["fc1.bias"], st.metrics.train_view(),
                                       st._fc_update() if st.fuse_fc1 else None),
          "cnn_bwd": lambda: C.cnn_bwd(st.xg, P["conv1.weight"], P["conv1.bias"], st.dpool, st.pmask,
                                       st.w2t, B, ipb, st.conv_slab, None, bands, st.a1g, st.xng),
          "conv_reduce": lambda: C.conv_reduce(st.conv_slab, nblk, G["conv2.weight"],
                                               G["conv2.bias"], G["conv1.weight"], G["conv1.bias"]),
          # the training step's update: the slab-fused launch at world size 1
          "optim": (lambda: st.launch_optimizer(st._fused_segments(nblk)))
                   if st.fuse_conv_reduce else (lambda: st.launch_optimizer()),
      }
      tot = 0.0
      line = []
      for name, fn in ks.items():
          us = timeit(fn)
          tot += us
          line.append(f"{name}={us:.1f}")
      st.ctr.zero_()   # each step advances the data counter (rows are clamped past the epoch)
      step = timeit(lambda: st._train_impl(B), 8)
      print(f"B={B:5d} S={S} ipb={ipb} bands={bands} " + " ".join(line) + f" | sum={tot:.1f}us step={step:.1f}us "
            f"-> {B / step * 1e6 / 1e6:.2f}M img/s", flush=True)


if __name__ == "__main__":
    main()
