"""Does a HIP-graph capture that records nothing end cleanly on this stack?  (The capture-misuse
test raises before any kernel of its backward is enqueued; if capture_end then segfaults, the
cause is the empty graph, not the refused launch.)  Exit 0: clean; the parent reads the signal."""
import torch

g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        pass
torch.cuda.synchronize()
print("empty capture ended cleanly")
