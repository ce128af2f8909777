"""CPU oracle for the PageRank / BFS / SSSP / Louvain hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker (or the timed CPU baseline), never
as the thing measured or shipped.  The product path (``cugraph-forked_amd``)
never imports this package and fails loudly when its HIP library is missing.

The oracle is a plain numpy restatement of the reference algorithms
(RAPIDS cuGraph 22.10, mounted read-only at ``/root/reference``):

* ``graph``    -- edge list -> renumbered CSR/CSC, following
                  ``cpp/src/structure/create_graph_from_edgelist_impl.cuh:557-776``
                  and ``cpp/src/structure/renumber_edgelist_impl.cuh:95-452``.
* ``pagerank`` -- ``cpp/src/link_analysis/pagerank_impl.cuh:48-293``.
* ``bfs``      -- ``cpp/src/traversal/bfs_impl.cuh:94-287``.
* ``sssp``     -- ``cpp/src/traversal/sssp_impl.cuh:79-270``.
* ``louvain``  -- ``cpp/src/community/louvain_impl.cuh:46-255`` and
                  ``cpp/src/community/detail/common_methods.cuh:49-382``.
* ``rmat``     -- our own counter-based Graph500 R-MAT generator; the HIP
                  generator in ``cugraph-forked_amd/csrc/rmat.hip`` is its twin.

Parity pinning: every restatement is checked (``tests/test_oracle_golden.py``)
against the golden vectors the reference's own tests hold
(``cpp/tests/c_api/*_test.c``, ``python/pylibcugraph/pylibcugraph/tests``,
``cpp/tests/community/louvain_test.cpp``) and against NetworkX 3.4.2, the
reference's own Python test oracle.  The reference itself cannot be built or
imported here ("Oracle"), so no ``oracle/_ref`` exists.
"""
