"""cugraph.generators.rmat (reference python/cugraph/cugraph/generators/rmat.py)
over the device generator of this build (definition: oracle/rmat.py)."""
from __future__ import annotations


def rmat(scale, num_edges, a=0.57, b=0.19, c=0.19, seed=42, clip_and_flip=False, scramble_vertex_ids=False,
         return_type=None, mg=False, create_using=None):
    """Returns a pandas DataFrame ['src', 'dst'] (or a Graph when create_using is a
    cugraph graph class / instance)."""
    import pandas as pd
    import pylibcugraph as p
    if mg:
        raise NotImplementedError("mg=True is not supported by this build; use MGGraph directly")
    h = p.ResourceHandle()
    s, d = p.generators.generate_rmat_edgelist(h, scale, num_edges, a, b, c, seed, clip_and_flip,
                                               scramble_vertex_ids)
    df = pd.DataFrame({"src": s.cpu().numpy(), "dst": d.cpu().numpy()})
    if create_using is None:
        return df
    G = create_using() if isinstance(create_using, type) else create_using
    G.from_pandas_edgelist(df, "src", "dst")
    return G
