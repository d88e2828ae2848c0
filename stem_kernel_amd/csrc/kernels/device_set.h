// Device-resident packed example set (shared by the HIP kernels and the host
// packer).  One flat SoA buffer per field, examples concatenated.
//
// DAG part: only NON-LEAF nodes are stored (leaves are implicit: G0 at a
// leaf row/column is a closed form, see dag_stem.hip), renumbered in LEVEL
// order: level 0 = loop nodes (single leaf child), level k>0 = stems whose
// deepest non-leaf child is at level k-1.  Level order is a topological order
// (children first) and makes every level a contiguous node range.
#pragma once
#include <cstdint>

namespace sk {


// x-role row header (post-order row r of an example)
struct XRow {
  uint32_t a;    // n_ch:8 | n_bpf:8 | loop leaf-edge gaps:16
  uint32_t b;    // len:16 | out slot:16 (0xffff = row never read)
  uint32_t c;    // bpf_beg_local:16 | code of first bp entry:8
  float w;       // node weight
  float nbp;     // profile gap count at node.first
  float bp0;     // p of the first bp entry
  double P;      // root->node path count
};
static_assert(sizeof(XRow) == 32, "XRow is one 32-byte scalar load");

struct DevSet {
  int32_t n_examples = 0;
  // per example (n_examples entries; *_base are absolute indices)
  const int32_t* ex_nl = nullptr;         // non-leaf node count
  const int32_t* ex_node_base = nullptr;  // into nd_* arrays
  const int32_t* ex_edge_base = nullptr;  // into ed_* arrays
  const int32_t* ex_bpf_base = nullptr;   // into bpf_* arrays
  const int32_t* ex_lvl_base = nullptr;   // into lvl (n_levels+1 offsets, local)
  const int32_t* ex_nlev = nullptr;       // number of levels
  const float* ex_nseqs = nullptr;        // ProfileSequence::n_seqs
  const int32_t* ex_len = nullptr;        // aligned length
  const int32_t* ex_pos_base = nullptr;   // into pos_* arrays
  // per non-leaf node (level order)
  const uint32_t* nd_a = nullptr;  // edge_beg_local:16 | n_edges:8 | n_bpf:8  (non-leaf edges only)
  const uint32_t* nd_b = nullptr;  // len(last-first):16 | bpf_beg_local:16
  const uint32_t* nd_c = nullptr;  // loop nodes: gaps of the leaf edge (else 0)
  const float* nd_w = nullptr;     // node weight (loop_profile(i)*loop_profile(j))
  const float* nd_nbp = nullptr;   // profile gap count at node.first
  const double* nd_P = nullptr;    // sum over roots of #paths root->node
  // non-leaf edges of stem nodes, node-major in reference list order; level
  // order of nodes makes every level's edges one contiguous range
  const uint2* ed = nullptr;  // {child_local | gaps<<16, parent_local}
  // per bp-frequency entry
  const uint32_t* bpf_code = nullptr;  // a*4+b
  const float* bpf_p = nullptr;
  // level offsets (local node index)
  const int32_t* lvl = nullptr;
  // per aligned position (string kernel)
  const float4* pos_prof = nullptr;  // ProfileSequence columns A,C,G,U
  const float* pos_w = nullptr;      // fill_weight (empty -> string kernel unweighted)
  const int32_t* ex_has_w = nullptr;
  const uint8_t* pos_chr = nullptr;  // raw characters of row 0 (naive string kernel)
  const float4* pos_lru = nullptr;   // BPLA fill_weight: sqrt p_left, p_right, p_unpair, 0
  // x-role schedule, in the reference's post-order (children first, a row's
  // last parent soon after it).  Row r of example e is xr_*[ex_node_base[e]+r];
  // its children are xr_ch[ex_xch_base[e] + sum of earlier rows' n_ch ...].
  const int32_t* ex_nslots = nullptr;   // recycled HBM row slots this example needs
  const int32_t* ex_xch_base = nullptr; // into xr_ch
  const XRow* xrow = nullptr;       // one 32-B record per row (wave-uniform scalar load)
  const uint32_t* xr_node = nullptr;  // level-order node id (for nd_SL)
  const uint32_t* xr_ch = nullptr;  // per child edge: child slot:16 | gaps:16
  // y role of the stem kernel: non-leaf nodes sorted by length (sorted
  // ids), edges packed child:11|parent:11|gaps:10 in sorted ids
  const uint32_t* yn_a = nullptr;   // first edge in ye2:16 | n_edges:8 | n_bpf:8
  const uint32_t* yn_b = nullptr;   // len:16 | bpf_beg:16
  const float* yn_w = nullptr;
  const float* yn_nbp = nullptr;
  const double* yn_P = nullptr;
  const uint32_t* yn_c = nullptr;   // loop leaf-edge gaps:16 | bc0:4 | single-entry flag @24
  const float* yn_p0 = nullptr;     // p of the first bp-freq entry
  const uint4* yrec = nullptr;      // node record {yn_a, yn_c, w, p0} (16 B)
  const uint32_t* ye2 = nullptr;    // edges node-major (sorted ids), ex_edge_base[e] per example
  // IY sweep schedule: ex_nch[e] chunks of 64 records child:11 | parent:11 |
  // gaps:10 from ysc[64 * ex_ysc_base[e]] (dummy records: child == parent);
  // ycs[ex_ycs_base[e] + v], v <= max node length + 1: first chunk whose
  // prefix maximum of the children's lengths reaches v
  const uint32_t* ysc = nullptr;
  const int32_t* ex_ysc_base = nullptr;
  const int32_t* ex_nch = nullptr;
  const int32_t* ycs = nullptr;
  const int32_t* ex_ycs_base = nullptr;
  // Gamma schedule (dag_stem.hip): the x rows in post-order without the gamma
  // rows (x loop rows with one bp-frequency entry and no gap column, whose G0
  // row is g^lg pf Gamma_{code,len}(y)); a child record with bit 15 set is a
  // gamma child (low bits: gamma index), its weight factors in xg_clg
  // (loop leaf gaps) and xg_cpf (pf); gr_* lists the gamma rows for their K
  // terms.  gam_key[g] = code:16 | len:16, n_gam keys over the set.
  const XRow* xgrow = nullptr;
  const uint32_t* xg_node = nullptr;
  const uint32_t* xg_ch = nullptr;
  const uint32_t* xg_clg = nullptr;
  const float* xg_cpf = nullptr;
  const int32_t* ex_xg_base = nullptr;
  const int32_t* ex_nlxg = nullptr;
  const int32_t* ex_xgch_base = nullptr;
  const uint32_t* gr_info = nullptr;  // gamma index:16 | loop leaf gaps:16
  const float* gr_pf = nullptr;
  const double* gr_P = nullptr;
  const int32_t* ex_gr_base = nullptr;  // n_examples + 1 entries
  const int32_t* ex_gapless = nullptr;  // y role: no gap column in any non-leaf node
  const uint32_t* gam_key = nullptr;
  int32_t n_gam = 0;
  // phi rows (combination rows, flag bit 31 of XRow.c): child record bit 14
  // = a Phi table row (low bits: phi index); xg_cty per record its weight
  // recipe (0 g^gaps; 1 gamma child g^gaps g^lg pf; 2 Phi component
  // pf_p g^gaps g^lg pf_c; 3 Gamma_{code,len} component pf_p xSL_p; 4 Gamma
  // component of a child gap2 w_p g^gaps g^lg pf_c); gra_* the rows'
  // Gamma_{code,len} K terms (gamma index, gamma-schedule row); phk_idx per
  // example the phi index of each type-2 record, in record order; phi key t =
  // (phi_al[t] = code:16 | len:16, phi_g[t] = gamma index of the child key)
  const uint8_t* xg_cty = nullptr;
  const uint32_t* gra_gidx = nullptr;
  const uint32_t* gra_row = nullptr;
  const int32_t* ex_gra_base = nullptr;  // n_examples + 1
  const uint32_t* phk_idx = nullptr;
  const int32_t* ex_phk_base = nullptr;  // n_examples + 1
  const uint32_t* phi_al = nullptr;
  const uint32_t* phi_g = nullptr;
  int32_t n_phi = 0;
  // maxima over the set
  int32_t max_nl = 0, max_edges = 0, max_bpf = 0, max_nlev = 0, max_len = 0, max_slots = 0;
  int32_t max_nch = 0;
  int64_t total_nodes = 0;
};

// Per-call, parameter-dependent node values (computed on device by sk_prep).
struct DevParamNodes {
  double* nd_L = nullptr;   // G0 at (node, any y-leaf column), level order
  double* nd_SL = nullptr;  // sum_e g^gaps(e) * L[child(e)], level order
  double* xr_SL = nullptr;  // nd_SL in x-row (post-)order
  // gamma schedule: nd_SL per row, child weights g^gaps (x g^lg pf for a
  // gamma child), and per example sum over its gamma rows of P g^lg pf by
  // gamma index (n_examples x n_gam)
  double* xg_SL = nullptr;
  double* xg_chw = nullptr;
  double* gam_h = nullptr;
  double* xr_chw = nullptr;  // x schedule child weights g^gaps
  double* phk_w = nullptr;   // per phi component: P_p times its record weight (K terms)
};

}  // namespace sk
