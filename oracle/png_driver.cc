// Test-infrastructure driver (not product code): the reference CLI's PNG
// reader, ReadPNG (guetzli/guetzli.cc:51-156: libpng with PACKING | EXPAND |
// STRIP_16, alpha blended on black), compiled from /root/reference and run
// on the PNG fixtures so that the product's PNG decoder is pinned to it.
//
//   png_driver IN.png OUT.rgb      writes W H on stdout, the RGB8 to OUT.rgb;
//                                  exit 1 when ReadPNG fails
//
// guetzli.cc is compiled in this TU (its ReadPNG lives in an anonymous
// namespace) with its main() renamed.
#define main guetzli_cli_main
#include "guetzli/guetzli.cc"
#undef main

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s IN.png OUT.rgb\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::string data;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, n);
  fclose(f);
  int w = 0, h = 0;
  std::vector<uint8_t> rgb;
  if (!ReadPNG(data, &w, &h, &rgb)) return 1;
  FILE* o = fopen(argv[2], "wb");
  if (!o || fwrite(rgb.data(), 1, rgb.size(), o) != rgb.size()) return 2;
  fclose(o);
  printf("%d %d\n", w, h);
  return 0;
}
