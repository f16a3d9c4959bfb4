// C++ drop-in check: the ITK-shaped facade (include/mad_itk.hpp) used exactly like
// test/itk2DDiffusionTest_WJ.cxx:47-109 uses the reference filter.
//   facade_test host   -> host-only calls (no GPU): defaults + depth rule
//   facade_test run    -> 2D filter run on the GPU, prints the output checksum
//   facade_test run bench -> the same with SetBenchmark(true) (the reference's -DBENCHMARK build):
//                         2 nu + 1 "relres_seconds" lines per V-cycle in ./benchmark.txt
//   facade_test ved    -> VEDMultigridImageFilter on a short 3D volume with a bright tube,
//                         set up like test/itkVEDTest_GS.cxx:46-95
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>

#include "mad_itk.hpp"

using ImageType = mad::itkshim::Image<float, 2>;
using FilterType = mad::MultigridAnisotropicDiffusionImageFilter<
    ImageType, ImageType, mad::MultigridWeightedJacobiSmoother<2>>;

using VolumeType = mad::itkshim::Image<short, 3>;
using VedType = mad::VEDMultigridImageFilter<VolumeType, VolumeType, mad::MultigridGaussSeidelSmoother<3>>;

static int run_ved() {
  auto input = VolumeType::New();
  input->SetRegions({40, 36, 32});
  input->Allocate();
  input->SetSpacing({0.3125, 0.3125, 0.5});
  short* p = input->GetBufferPointer();
  for (int z = 0; z < 32; ++z)
    for (int y = 0; y < 36; ++y)
      for (int x = 0; x < 40; ++x) {
        const double d2 = (x - 20.0) * (x - 20.0) + (y - 18.0) * (y - 18.0);
        p[(z * 36 + y) * 40 + x] = (short)(200.0 * std::exp(-d2 / 18.0) + ((x * 7 + y * 3 + z) % 11));
      }
  auto filter = VedType::New();
  filter->SetCycle(VedType::VCYCLE);
  filter->SetDiffusionIterationsPerGrid(3);
  filter->SetInput(input.get());
  filter->SetScales({0.300, 0.482, 0.775, 1.245, 2.000});
  filter->SetAlpha(0.5);
  filter->SetBeta(0.5);
  filter->SetGamma(5.);
  filter->SetEpsilon(0.01);
  filter->SetSensitivity(10.);
  filter->SetIterations(1);
  filter->SetTolerance(1e-10);
  filter->SetTimeStep(0.1);
  filter->SetDiffusionIterations(4);
  filter->SetOmega(1.5);
  filter->Update();
  auto out = filter->GetOutput();
  long sum = 0;
  for (int64_t i = 0; i < out->NumberOfPixels(); ++i) sum += out->GetBufferPointer()[i];
  std::printf("ved ok cycles=%u relres=%.3e checksum=%ld\n", filter->GetStats().total_cycles,
              filter->GetStats().last_relres, sum);
  return filter->GetStats().iterations == 1 && filter->GetStats().total_cycles >= 4 ? 0 : 5;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "ved") == 0) return run_ved();
  const bool run = argc > 1 && std::strcmp(argv[1], "run") == 0;
  const bool bench = run && argc > 2 && std::strcmp(argv[2], "bench") == 0;
  mad_desc d;
  mad_desc_init(&d);
  if (d.iterations_per_grid != 2 || d.max_cycles != 100 || d.time_step != 0.01) return 2;
  const int64_t sz[3] = {256, 256, 1};
  if (mad_max_depth(2, sz) != 5) return 3;
  if (!run) {
    std::printf("host ok\n");
    return 0;
  }
  auto input = ImageType::New();
  input->SetRegions({64, 48});
  input->Allocate();
  input->SetSpacing({1.0, 1.0});
  for (int64_t i = 0; i < input->NumberOfPixels(); ++i)
    input->GetBufferPointer()[i] = (float)(128.0 + 60.0 * std::sin(0.1 * (double)i));
  auto tensor = FilterType::InputTensorImageType::New();
  tensor->SetRegions({64, 48});
  tensor->Allocate();
  for (int64_t i = 0; i < tensor->NumberOfPixels(); ++i) {
    auto& t = tensor->GetBufferPointer()[i];
    t(0, 0) = 50.f;  // itk2DDiffusionTest_GS.cxx:65-70
    t(1, 1) = 30.f;
    t(0, 1) = 0.f;
  }
  auto filter = FilterType::New();
  filter->SetInput(input.get());
  filter->SetDiffusionTensor(tensor.get());
  filter->SetIterationsPerGrid(2);
  filter->SetTimeStep(0.1);
  filter->SetNumberOfSteps(1);
  filter->SetMaxCycles(100);
  filter->SetTolerance(1e-6);
  filter->SetCycle(FilterType::VCYCLE);
  if (bench) filter->SetBenchmark(true);
  filter->Update();
  if (bench) {
    const auto lines = filter->GetBenchmarkOutput();
    std::ifstream f("benchmark.txt");
    std::string ln;
    size_t nf = 0;
    while (std::getline(f, ln)) nf += ln.find('_') != std::string::npos;
    std::printf("benchmark lines=%zu file=%zu first=%s last=%s\n", lines.size(), nf,
                lines.empty() ? "" : lines.front().c_str(), lines.empty() ? "" : lines.back().c_str());
    if (lines.size() != 5u * filter->GetStats().total_cycles || nf != lines.size()) return 6;
  }
  double sum = 0.0;
  auto out = filter->GetOutput();
  for (int64_t i = 0; i < out->NumberOfPixels(); ++i) sum += out->GetBufferPointer()[i];
  std::printf("run ok cycles=%u relres=%.3e checksum=%.6f\n", filter->GetStats().total_cycles,
              filter->GetStats().last_relres, sum);
  return filter->GetStats().last_relres <= 1e-6 ? 0 : 4;
}
