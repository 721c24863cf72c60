"""Source rewriting helper used once per kernel file when the 16-bit MFMA operand type became a
template parameter (common.h HalfType); kept for reference with tools/isa_same.py, which checks
that the bf16 instantiations compile to the same instructions as before.

    rw = Rewriter(text)
    rw.kernel("vconv3x3_kernel", typedefs={"vgb8": 8, "vgb4": 4})   # adds `typename T16`
    text = rw.finish()
"""
import re


class Rewriter:
    def __init__(self, text):
        i = text.index("}  // namespace dsg")
        self.body, self.abi = text[:i], text[i:]

    def rep(self, a, b, count=1, where="body"):
        s = getattr(self, where)
        n = s.count(a)
        if n != count:
            raise AssertionError("expected %d x %r, found %d" % (count, a[:80], n))
        setattr(self, where, s.replace(a, b))

    def drop_typedef(self, name):
        self.body, n = re.subn(r"typedef __attribute__\(\(ext_vector_type\((\d+)\)\)\) __bf16 %s;\n" % name, "",
                               self.body)
        assert n == 1, name

    def kernel(self, name, typedefs=None):
        """Give function `name` a leading `typename T16` template parameter (merging with an existing
        template header) and, optionally, local typedefs of 16-bit vectors."""
        m = re.search(r"((?:template <([^\n]*)>\n)?)(?:__global__|__device__|static)[^\n]*?\b%s\(" % re.escape(name),
                      self.body)
        assert m, name
        hdr = m.group(1)
        if hdr:
            new_hdr = "template <typename T16, %s>\n" % m.group(2)
        else:
            new_hdr = "template <typename T16>\n"
        start = m.start()
        self.body = self.body[:start] + new_hdr + self.body[start + len(hdr):]
        if typedefs:
            j = self.body.index("{", self.body.index(name + "(", start))
            td = "".join("\n  typedef hx%d<T16> %s;" % (n, k) for k, n in typedefs.items())
            self.body = self.body[:j + 1] + td + self.body[j + 1:]

    def finish(self):
        b = self.body.replace("__bf16", "T16")
        b = re.sub(r"__builtin_amdgcn_mfma_f32_32x32x16_bf16\(([^;]*?), 0, 0, 0\)", r"mfma16(\1)", b)
        assert "__builtin_amdgcn_mfma_f32_32x32x16_bf16" not in b
        return b + self.abi
