"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the GraphCNNDropEdge hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package.  The product path (graph-representation-learning_amd/) must
never import it: a GPU result is only ever *checked* against it.

  oracle.hash       numpy restatement of the DropEdge / synthetic-graph hash
  oracle.dense_ref  numpy restatement of the reference's dense GraphConv and
                    GraphCNNDropEdge forward/backward (robust_gcn.py,
                    drop_robust_gcn.py)
  oracle.c_oracle   ctypes wrapper of grl_oracle.c (typed-CSR restatement,
                    OpenMP; also the CPU baseline)

Parity pin: tests/golden/*.npz, produced by the reference itself
(tests/golden/make_golden.py).
"""
