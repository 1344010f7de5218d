// JNodeTable storage modes (sheep_amd/lib/jnode.h): a tree built into a mapped .tre, reopened
// mapped in place, merged into a mapped table, and saved from both modes — the bytes equal the
// heap table's.  Host only: the merge is not called here (it runs on the GPU).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "jnode.h"

static std::string slurp(const char* f) {
  std::ifstream s(f, std::ios::binary);
  return std::string(std::istreambuf_iterator<char>(s), {});
}

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string dir = argv[1];
  const std::string a = dir + "/a.tre", b = dir + "/b.tre", c = dir + "/c.tre";
  std::vector<jnid_t> parent = {3, 6, 3, 6, 5, INVALID_JNID, INVALID_JNID};
  std::vector<esize_t> pst = {1, 2, 2, 1, 3, 0, 0};
  {
    JNodeTable heap(parent, pst);
    CHECK(!heap.mapped());
    heap.save(b.c_str());
  }
  {
    JNodeTable m(a.c_str(), (jnid_t)parent.size());  // created, all roots
    CHECK(m.mapped() && m.size() == parent.size());
    for (jnid_t i = 0; i < m.size(); ++i) CHECK(m.parent(i) == INVALID_JNID && m.pst_weight(i) == 0);
    m.assign(parent, pst);
    JNodeTable moved(std::move(m));  // the mapping moves with the table
    CHECK(moved.mapped() && !m.mapped());
  }  // unmapped: the header holds end_id
  CHECK(slurp(a.c_str()) == slurp(b.c_str()));
  {
    JNodeTable m(a.c_str());  // the open constructor maps it in place
    CHECK(m.mapped() && m.size() == 7);
    for (jnid_t i = 0; i < 7; ++i) CHECK(m.parent(i) == parent[i] && m.pst_weight(i) == pst[i]);
    CHECK(m.hasKids() && m.kids_end(6) - m.kids_begin(6) == 2 && m.kids_begin(6)[0] == 1 && m.kids_begin(6)[1] == 3);
    m.pst_weight(0) = 9;  // writes go to the file
    m.save(c.c_str());
  }
  std::string sa = slurp(a.c_str()), sc = slurp(c.c_str());
  CHECK(sa == sc && sa.size() == 4 + 7 * 8);
  JNodeTable r(a.c_str());
  CHECK(r.pst_weight(0) == 9);
  r.pst_weight(0) = 1;
  JNodeTable::Facts f(r);
  CHECK(f.root_cnt == 2 && f.edge_cnt == 9 && f.vert_cnt == 7);
  printf("ok\n");
  return 0;
}
