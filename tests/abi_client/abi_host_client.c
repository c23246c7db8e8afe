/*
 * abi_host_client.c — a plain C caller of libcda.so that uses the C ABI exactly as the cgo shim in
 * go/cda does: malloc'd (pageable) host buffers standing in for Go slices, flattened shares, roots as
 * 90-byte records, error details through cda_err_info.  Built by __graft_entry__.build() (gcc, against
 * include/cda.h); run by tests/test_abi_client.py on the GPU, which checks its outputs against
 * tests/golden/oracle_digests.json and mainnet block 408's data_hash.
 *
 *   abi_host_client <ods.bin> <k> <out_dir> [<blobs.bin>] [--proof <start> <end>] [--nodes] [--segments <segs.bin>]
 * writes <out_dir>/{eds,row_roots,col_roots,dah,parity,repaired,commitments}.bin and prints one status line.
 * With <blobs.bin> ([u32 n][n x 29-B namespace][(n + 1) x u64 data offsets][data]) it also computes the share
 * commitments of all n blobs in ONE cda_blob_commitments call -- ProcessProposal's pre-pass over every BlobTx of a
 * proposal (go/patches/0003) -- into <out_dir>/proposal_commitments.bin.
 * The calls go/cda's f1 / f3 bindings make (go/cda/proof.go, go/cda/square.go; go/patches/0005):
 *   --proof S E   pkg/proof NewShareInclusionProof of ODS shares [S, E) (cda_share_inclusion_proof) -> proof.bin:
 *                 cda_share_proof_info | row roots | leaf hashes | aunts | nmt start, end, count (i32) | nmt nodes |
 *                 data root, each section sized by the info (capacity k rows);
 *   --nodes       pkg/inclusion's subtree cacher: every node of every row / column tree and of the DAH tree
 *                 (cda_extend_commit_nodes) -> row_nodes.bin, col_nodes.bin, dah_nodes.bin;
 *   --segments F  square.Construct on the device from a host layout plan (cda_construct_extend_commit); F =
 *                 [u32 nseg][nseg x cda_share_segment][u64 data_len][data][u32 nres][nres x u32] ->
 *                 construct_ods.bin, construct_dah.bin.
 * Also checked in-process: Codec.Decode of an erased row, a wrapper tree root, the multi-device batch.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "cda.h"

static int write_file(const char* dir, const char* name, const void* p, size_t n) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  const size_t w = fwrite(p, 1, n, f);
  fclose(f);
  return w == n ? 0 : -1;
}

static int fail(const char* what, int rc, const cda_err_info* e) {
  fprintf(stderr, "%s: rc=%d (%s) axis=%d index=%d leaf=%d block=%d\n", what, rc, cda_strerror(rc),
          e ? e->axis : -1, e ? e->index : -1, e ? e->leaf : -1, e ? e->block : -1);
  return 1;
}

static uint8_t* read_all(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f || fseek(f, 0, SEEK_END) != 0) return NULL;
  const long sz = ftell(f);
  uint8_t* b = malloc((size_t)sz + 1);
  rewind(f);
  if (sz < 0 || fread(b, 1, (size_t)sz, f) != (size_t)sz) {
    fclose(f);
    free(b);
    return NULL;
  }
  fclose(f);
  *n = (size_t)sz;
  return b;
}

/* pkg/proof NewShareInclusionProof through cda_share_inclusion_proof (what go/cda.ShareInclusionProof binds) */
static int run_proof(cda_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t start, uint32_t end, const char* dir) {
  const uint32_t lg = (uint32_t)__builtin_ctz(2 * k), cap = k, naunts_max = lg + 1, max_nodes = 2 * lg;
  cda_share_proof_info info;
  uint8_t* rr = malloc((size_t)cap * CDA_NODE_SIZE);
  uint8_t* lh = malloc((size_t)cap * 32);
  uint8_t* au = malloc((size_t)cap * naunts_max * 32);
  int32_t* ns = malloc((size_t)cap * 4 * 3);
  uint8_t* nodes = malloc((size_t)cap * (max_nodes ? max_nodes : 1) * CDA_NODE_SIZE);
  uint8_t root[32];
  cda_err_info err;
  int rc = cda_share_inclusion_proof(ctx, k * k, CDA_SHARE_SIZE, ods, start, end, &info, rr, lh, au, ns, ns + cap,
                                     ns + 2 * cap, nodes, root, &err);
  if (rc) return fail("cda_share_inclusion_proof", rc, &err);
  char path[4096];
  snprintf(path, sizeof path, "%s/proof.bin", dir);
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  fwrite(&info, sizeof info, 1, f);
  fwrite(rr, CDA_NODE_SIZE, info.nrows, f);
  fwrite(lh, 32, info.nrows, f);
  for (uint32_t i = 0; i < info.nrows; i++) fwrite(au + (size_t)i * naunts_max * 32, 32, info.naunts, f);
  fwrite(ns, 4, info.nrows, f);
  fwrite(ns + cap, 4, info.nrows, f);
  fwrite(ns + 2 * cap, 4, info.nrows, f);
  for (uint32_t i = 0; i < info.nrows; i++)
    fwrite(nodes + (size_t)i * info.max_nodes * CDA_NODE_SIZE, CDA_NODE_SIZE, (size_t)ns[2 * cap + i], f);
  fwrite(root, 32, 1, f);
  fclose(f);
  free(rr), free(lh), free(au), free(ns), free(nodes);
  return 0;
}

/* every tree node the block path builds (cda_extend_commit_nodes; go/cda.ExtendCommitNodes) */
static int run_nodes(cda_ctx* ctx, const uint8_t* ods, uint32_t k, const uint8_t* dah_want, const char* dir) {
  const uint32_t w = 2 * k;
  const size_t tree_b = (size_t)w * (2 * w - 1) * CDA_NODE_SIZE;
  uint8_t* rn = malloc(tree_b);
  uint8_t* cn = malloc(tree_b);
  uint8_t* dn = malloc((size_t)(4 * w - 1) * 32);
  uint8_t* rows = malloc((size_t)w * CDA_NODE_SIZE);
  uint8_t* cols = malloc((size_t)w * CDA_NODE_SIZE);
  uint8_t dah[32];
  cda_err_info err;
  int rc = cda_extend_commit_nodes(ctx, k * k, CDA_SHARE_SIZE, ods, NULL, rows, cols, dah, rn, cn, dn, &err);
  if (rc) return fail("cda_extend_commit_nodes", rc, &err);
  if (memcmp(dah, dah_want, 32) != 0 || memcmp(dn + (size_t)(4 * w - 2) * 32, dah, 32) != 0) {
    fprintf(stderr, "node export DAH differs\n");
    return 1;
  }
  for (uint32_t t = 0; t < w; t++)  /* each tree's last node is its root */
    if (memcmp(rn + ((size_t)t * (2 * w - 1) + 2 * w - 2) * CDA_NODE_SIZE, rows + (size_t)t * CDA_NODE_SIZE, CDA_NODE_SIZE) ||
        memcmp(cn + ((size_t)t * (2 * w - 1) + 2 * w - 2) * CDA_NODE_SIZE, cols + (size_t)t * CDA_NODE_SIZE, CDA_NODE_SIZE)) {
      fprintf(stderr, "exported root of tree %u differs\n", t);
      return 1;
    }
  if (write_file(dir, "row_nodes.bin", rn, tree_b) || write_file(dir, "col_nodes.bin", cn, tree_b) ||
      write_file(dir, "dah_nodes.bin", dn, (size_t)(4 * w - 1) * 32))
    return 1;
  free(rn), free(cn), free(dn), free(rows), free(cols);
  return 0;
}

/* square.Construct + ExtendShares + NewDataAvailabilityHeader from a layout plan (cda_construct_extend_commit;
 * go/cda.ConstructExtendCommit) */
static int run_segments(cda_ctx* ctx, uint32_t k, const char* path, const char* dir) {
  size_t n = 0;
  uint8_t* b = read_all(path, &n);
  if (!b || n < 4) return 2;
  uint32_t nseg;
  memcpy(&nseg, b, 4);
  const cda_share_segment* segs = (const cda_share_segment*)(b + 4);
  size_t at = 4 + (size_t)nseg * sizeof(cda_share_segment);
  uint64_t dlen;
  memcpy(&dlen, b + at, 8);
  const uint8_t* data = b + at + 8;
  at += 8 + dlen;
  uint32_t nres;
  memcpy(&nres, b + at, 4);
  uint32_t* res = malloc(((size_t)nres + 1) * 4);
  memcpy(res, b + at + 4, (size_t)nres * 4);
  const uint32_t w = 2 * k;
  uint8_t* ods = malloc((size_t)k * k * CDA_SHARE_SIZE);
  uint8_t* rows = malloc((size_t)w * CDA_NODE_SIZE);
  uint8_t* cols = malloc((size_t)w * CDA_NODE_SIZE);
  uint8_t dah[32];
  cda_err_info err;
  int rc = cda_construct_extend_commit(ctx, k, nseg, segs, data, dlen, res, nres, ods, NULL, rows, cols, dah, &err);
  if (rc) return fail("cda_construct_extend_commit", rc, &err);
  if (write_file(dir, "construct_ods.bin", ods, (size_t)k * k * CDA_SHARE_SIZE) ||
      write_file(dir, "construct_dah.bin", dah, 32))
    return 1;
  free(b), free(res), free(ods), free(rows), free(cols);
  return 0;
}

int main(int argc, char** argv) {
  const char* blobs_path = NULL;
  const char* segs_path = NULL;
  int want_nodes = 0, want_proof = 0;
  uint32_t p_start = 0, p_end = 0;
  for (int a = 4; a < argc; a++) {
    if (!strcmp(argv[a], "--proof") && a + 2 < argc) {
      want_proof = 1;
      p_start = (uint32_t)atoi(argv[++a]);
      p_end = (uint32_t)atoi(argv[++a]);
    } else if (!strcmp(argv[a], "--nodes")) {
      want_nodes = 1;
    } else if (!strcmp(argv[a], "--segments") && a + 1 < argc) {
      segs_path = argv[++a];
    } else if (a == 4 && strncmp(argv[a], "--", 2) != 0) {
      blobs_path = argv[a];
    } else {
      argc = 0;
      break;
    }
  }
  if (argc < 4) {
    fprintf(stderr, "usage: %s <ods.bin> <k> <out_dir> [<blobs.bin>] [--proof S E] [--nodes] [--segments F]\n",
            argv[0]);
    return 2;
  }
  const uint32_t k = (uint32_t)atoi(argv[2]), w = 2 * k, count = k * k;
  const size_t S = CDA_SHARE_SIZE;
  uint8_t* ods = malloc((size_t)count * S);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(ods, 1, (size_t)count * S, f) != (size_t)count * S) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  fclose(f);
  cda_ctx* ctx = NULL;
  int rc = cda_init(0, &ctx);
  if (rc) return fail("cda_init", rc, NULL);

  /* da.ExtendShares + NewDataAvailabilityHeader: one call */
  uint8_t* eds = malloc((size_t)w * w * S);
  uint8_t* rows = malloc((size_t)w * CDA_NODE_SIZE);
  uint8_t* cols = malloc((size_t)w * CDA_NODE_SIZE);
  uint8_t dah[32];
  cda_err_info err;
  rc = cda_extend_commit(ctx, count, (uint32_t)S, ods, eds, rows, cols, dah, &err);
  if (rc) return fail("cda_extend_commit", rc, &err);

  /* go/cda ExtendShares' call: the shares flattened into Q0 of a page-locked EDS buffer, extended in place
     (cda_host_register, cda_extend_commit_eds); the same square, roots and DAH */
  {
    uint8_t* ip = malloc((size_t)w * w * S);
    memset(ip, 0xC3, (size_t)w * w * S);
    for (uint32_t r = 0; r < k; r++) memcpy(ip + (size_t)r * w * S, ods + (size_t)r * k * S, (size_t)k * S);
    rc = cda_host_register(ctx, ip, (size_t)w * w * S);
    if (rc) return fail("cda_host_register", rc, NULL);
    uint8_t* r2 = malloc((size_t)w * CDA_NODE_SIZE);
    uint8_t* c2 = malloc((size_t)w * CDA_NODE_SIZE);
    uint8_t d2[32];
    rc = cda_extend_commit_eds(ctx, k, ip, r2, c2, d2, &err);
    if (rc) return fail("cda_extend_commit_eds", rc, &err);
    if (memcmp(ip, eds, (size_t)w * w * S) || memcmp(r2, rows, (size_t)w * CDA_NODE_SIZE) ||
        memcmp(c2, cols, (size_t)w * CDA_NODE_SIZE) || memcmp(d2, dah, 32)) {
      fprintf(stderr, "cda_extend_commit_eds differs from cda_extend_commit\n");
      return 1;
    }
    rc = cda_host_unregister(ctx, ip);
    if (rc) return fail("cda_host_unregister", rc, NULL);
    free(ip);
    free(r2);
    free(c2);
  }

  /* rsmt2d.Codec.Encode of ODS row 0 (the same bytes as EDS row 0, columns k..2k-1) */
  uint8_t* parity = malloc((size_t)k * S);
  rc = cda_rs_encode(ctx, k, (uint32_t)S, ods, parity);
  if (rc) return fail("cda_rs_encode", rc, NULL);
  if (memcmp(parity, eds + (size_t)k * S, (size_t)k * S) != 0) {
    fprintf(stderr, "codec parity differs from EDS row 0\n");
    return 1;
  }

  /* Repair from Q0 alone (the quarter of the square a light node must be able to rebuild from) */
  uint8_t* damaged = malloc((size_t)w * w * S);
  uint8_t* present = malloc((size_t)w * w);
  memcpy(damaged, eds, (size_t)w * w * S);
  for (uint32_t r = 0; r < w; r++)
    for (uint32_t c = 0; c < w; c++) {
      present[r * w + c] = (r < k && c < k) ? 1 : 0;
      if (!present[r * w + c]) memset(damaged + ((size_t)r * w + c) * S, 0, S);
    }
  rc = cda_repair(ctx, k, damaged, present, rows, cols, &err);
  if (rc) return fail("cda_repair", rc, &err);
  for (uint32_t i = 0; i < w * w; i++)
    if (!present[i]) {
      fprintf(stderr, "cell %u still missing after repair\n", i);
      return 1;
    }

  /* batch of three copies through the pipelined host path: same DAH each */
  uint8_t* ods3 = malloc((size_t)3 * count * S);
  for (int b = 0; b < 3; b++) memcpy(ods3 + (size_t)b * count * S, ods, (size_t)count * S);
  uint8_t* rows3 = malloc((size_t)3 * w * CDA_NODE_SIZE);
  uint8_t* cols3 = malloc((size_t)3 * w * CDA_NODE_SIZE);
  uint8_t dah3[96];
  rc = cda_extend_commit_batch(ctx, k, 3, ods3, NULL, rows3, cols3, dah3, &err);
  if (rc) return fail("cda_extend_commit_batch", rc, &err);
  for (int b = 0; b < 3; b++)
    if (memcmp(dah3 + 32 * b, dah, 32) != 0) {
      fprintf(stderr, "batch block %d DAH differs\n", b);
      return 1;
    }

  /* rsmt2d.Codec.Decode of EDS row 0 with every other shard erased (k of 2k present) */
  uint8_t* cw = malloc((size_t)w * S);
  uint8_t* cw_present = malloc(w);
  memcpy(cw, eds, (size_t)w * S);
  for (uint32_t i = 0; i < w; i++) {
    cw_present[i] = (uint8_t)(i % 2 == 0);
    if (!cw_present[i]) memset(cw + (size_t)i * S, 0xEE, S);
  }
  rc = cda_rs_decode(ctx, k, (uint32_t)S, cw, cw_present);
  if (rc) return fail("cda_rs_decode", rc, NULL);
  if (memcmp(cw, eds, (size_t)w * S) != 0) {
    fprintf(stderr, "decoded row 0 differs from the EDS\n");
    return 1;
  }

  /* wrapper.NewConstructor(k)(Row, 0): push row 0's 2k cells, Root() == the block path's row root 0 */
  uint8_t root[CDA_NODE_SIZE];
  rc = cda_nmt_axis_root(ctx, k, 0, w, (uint32_t)S, eds, root, &err);
  if (rc) return fail("cda_nmt_axis_root", rc, &err);
  if (memcmp(root, rows, CDA_NODE_SIZE) != 0) {
    fprintf(stderr, "axis root differs from row root 0\n");
    return 1;
  }

  /* inclusion.CreateCommitments over two blobs cut from the ODS bytes (namespace = share 0's) */
  const uint64_t tot = (uint64_t)count * S, b1 = tot / 2 < 1000 ? tot / 2 : 1000, b2 = b1 + 5000 < tot ? b1 + 5000 : tot;
  const uint64_t offs[3] = {0, b1, b2};
  uint8_t ns2[2 * CDA_NAMESPACE_SIZE];
  memcpy(ns2, ods, CDA_NAMESPACE_SIZE);
  memcpy(ns2 + CDA_NAMESPACE_SIZE, ods, CDA_NAMESPACE_SIZE);
  uint8_t commitments[64];
  rc = cda_blob_commitments(ctx, 2, ns2, ods, offs, NULL, 64, commitments, &err);
  if (rc) return fail("cda_blob_commitments", rc, &err);

  /* ProcessProposal's pre-pass: every blob of a proposal in one call */
  if (blobs_path) {
    FILE* bf = fopen(blobs_path, "rb");
    if (!bf || fseek(bf, 0, SEEK_END) != 0) {
      fprintf(stderr, "cannot read %s\n", blobs_path);
      return 2;
    }
    const long bsz = ftell(bf);
    uint8_t* bb = malloc((size_t)bsz + 1);
    rewind(bf);
    if (bsz < 4 || fread(bb, 1, (size_t)bsz, bf) != (size_t)bsz) {
      fprintf(stderr, "cannot read %s\n", blobs_path);
      return 2;
    }
    fclose(bf);
    uint32_t nb;
    memcpy(&nb, bb, 4);
    const uint8_t* bns = bb + 4;
    uint64_t* boffs = malloc(((size_t)nb + 1) * 8);
    memcpy(boffs, bns + (size_t)nb * CDA_NAMESPACE_SIZE, ((size_t)nb + 1) * 8);
    const uint8_t* bdata = bns + (size_t)nb * CDA_NAMESPACE_SIZE + ((size_t)nb + 1) * 8;
    uint8_t* pc = malloc((size_t)nb * 32);
    rc = cda_blob_commitments(ctx, nb, bns, bdata, boffs, NULL, 64, pc, &err);
    if (rc) return fail("cda_blob_commitments (proposal)", rc, &err);
    if (write_file(argv[3], "proposal_commitments.bin", pc, (size_t)nb * 32)) return 1;
    free(pc);
    free(boffs);
    free(bb);
  }

  /* the multi-device handle over every visible GPU: two blocks, same DAH each */
  cda_multi* multi = NULL;
  rc = cda_multi_init(0, &multi);
  if (rc) return fail("cda_multi_init", rc, NULL);
  uint8_t dahm[64];
  rc = cda_multi_extend_commit_batch(multi, k, 2, ods3, NULL, rows3, cols3, dahm, &err);
  if (rc) return fail("cda_multi_extend_commit_batch", rc, &err);
  if (memcmp(dahm, dah, 32) != 0 || memcmp(dahm + 32, dah, 32) != 0) {
    fprintf(stderr, "multi-device DAH differs\n");
    return 1;
  }
  /* one square split over the same devices (C5): same roots and DAH as the single-device call */
  rc = cda_multi_extend_commit_split(multi, k, ods, NULL, rows3, cols3, dahm, &err);
  if (rc) return fail("cda_multi_extend_commit_split", rc, &err);
  if (memcmp(dahm, dah, 32) != 0 || memcmp(rows3, rows, (size_t)w * CDA_NODE_SIZE) != 0 ||
      memcmp(cols3, cols, (size_t)w * CDA_NODE_SIZE) != 0) {
    fprintf(stderr, "split DAH / roots differ\n");
    return 1;
  }
  cda_multi_free(multi);

  if (want_proof && (rc = run_proof(ctx, ods, k, p_start, p_end, argv[3]))) return rc;
  if (want_nodes && (rc = run_nodes(ctx, ods, k, dah, argv[3]))) return rc;
  if (segs_path && (rc = run_segments(ctx, k, segs_path, argv[3]))) return rc;

  if (write_file(argv[3], "commitments.bin", commitments, sizeof commitments) ||
      write_file(argv[3], "eds.bin", eds, (size_t)w * w * S) || write_file(argv[3], "row_roots.bin", rows, (size_t)w * CDA_NODE_SIZE) ||
      write_file(argv[3], "col_roots.bin", cols, (size_t)w * CDA_NODE_SIZE) || write_file(argv[3], "dah.bin", dah, 32) ||
      write_file(argv[3], "parity.bin", parity, (size_t)k * S) || write_file(argv[3], "repaired.bin", damaged, (size_t)w * w * S)) {
    fprintf(stderr, "cannot write outputs\n");
    return 1;
  }
  printf("abi_host_client ok k=%u dah=", k);
  for (int i = 0; i < 32; i++) printf("%02x", dah[i]);
  printf("\n");
  cda_free(ctx);
  free(ods); free(eds); free(rows); free(cols); free(parity); free(damaged); free(present);
  free(ods3); free(rows3); free(cols3); free(cw); free(cw_present);
#if defined(__has_feature)
#if __has_feature(address_sanitizer)
  /* The AddressSanitizer build (make asan) leaves without the HIP runtime's exit-time teardown: there the ASan
     runtime's interception of HSA memory trips its own CHECK ("dev_runtime_unloaded_", inside libhsa-runtime64's
     destructors, after every libcda call has returned and cda_free has run) -- a sanitizer / runtime interaction,
     not a libcda access. */
  fflush(stdout);
  fflush(stderr);
  _exit(0);
#endif
#endif
  return 0;
}
